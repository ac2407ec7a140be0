# A/B of the v3 fused exact assign modes (+ exact-mode GPU tests on the new ABI)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5a}
timeout -k 10 400 python3 -u tools/kbench_v3.py --modes ${MODES:-v2,0,16,18,24,17,20,v2} > gpurun_out/${P}_v3ab.log 2>&1 || { tail -30 gpurun_out/${P}_v3ab.log; exit 1; }
cat gpurun_out/${P}_v3ab.log | grep mode
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kmeans_exact.py > gpurun_out/${P}_exact_tests.log 2>&1; rc=$?; tail -5 gpurun_out/${P}_exact_tests.log; exit $rc

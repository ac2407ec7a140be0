set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kmeans_exact.py tests/test_gpu_cluster.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_exact.log 2>&1; rc=$?; grep -E "PASSED|FAILED|agreement|Error" gpurun_out/pytest_exact.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/kmeans_fidelity.py --points 10000000 --iters 3 --out gpurun_out/kmeans_fidelity.json > gpurun_out/fidelity.log 2>&1; rc=$?; tail -4 gpurun_out/fidelity.log | cut -c1-1200; exit $rc

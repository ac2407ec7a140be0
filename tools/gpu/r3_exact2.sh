# round 3: exact-mode refine: the Elkan scan's work (neighbour distances per
# scan, full scans) at neighbour lists of 256 and 1024, and the exact tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3u}
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_exact_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_exact_tests.txt; exit 1; }
grep -E "agreement|passed|failed" gpurun_out/${P}_exact_tests.txt
for L in 256; do
  timeout -k 10 150 python tools/kbench_exact.py --nbr $L > gpurun_out/${P}_kbench_exact_$L.json 2> gpurun_out/${P}_kbench_exact_$L.err || { grep -v amdgpu.ids gpurun_out/${P}_kbench_exact_$L.err | tail -20; exit 1; }
  cat gpurun_out/${P}_kbench_exact_$L.json
done

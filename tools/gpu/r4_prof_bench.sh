# exact-mode tests, then the default bench (worker mode) under the kernel tracer
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4v}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -2
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
tail -1 gpurun_out/${P}_bench.json | cut -c1-250
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
grep '"metric"' gpurun_out/${P}_prof.log | cut -c1-200
ls gpurun_out/${P}_prof

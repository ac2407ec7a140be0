# round 4: fp16 exact mode — numerics tests, kernel micro-bench (f16 vs bf16), exact bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4f}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed|agreement" gpurun_out/${P}_tests.txt | tail -8
timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { tail -20 gpurun_out/${P}_kbench_exact.err; exit 1; }
cat gpurun_out/${P}_kbench_exact.json
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { tail -20 gpurun_out/${P}_bench_exact.err; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | cut -c1-400

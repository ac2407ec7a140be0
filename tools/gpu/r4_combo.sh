# exact-mode tests + kernel bench + exact bench, TeraSort GPU tests (out-of-core, output)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4p}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py tests/test_terasort.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -3
timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { tail -20 gpurun_out/${P}_kbench_exact.err; exit 1; }
cut -c1-500 gpurun_out/${P}_kbench_exact.json
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { tail -20 gpurun_out/${P}_bench_exact.err; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | cut -c1-300
HBMR_EXACT_EPI=top3 timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench_top3.json 2>&1 || { tail -20 gpurun_out/${P}_kbench_top3.json; exit 1; }
cut -c1-300 gpurun_out/${P}_kbench_top3.json

# exact-mode GPU tests, default bench, then the in-process kernel/host timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4y}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py tests/test_terasort.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -2
timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { tail -20 gpurun_out/${P}_kbench_exact.err; exit 1; }
cut -c1-600 gpurun_out/${P}_kbench_exact.json
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
tail -1 gpurun_out/${P}_bench.json | cut -c1-300
timeout -k 10 300 python bench.py --gpu-slots 1 --steps 10 --warmup 3 > gpurun_out/${P}_bench_1slot.json 2> gpurun_out/${P}_bench_1slot.err || { tail -20 gpurun_out/${P}_bench_1slot.err; exit 1; }
tail -1 gpurun_out/${P}_bench_1slot.json | cut -c1-200
timeout -k 10 300 python bench.py --steps 10 --warmup 3 -D hbmr.gpu.batch.taper=false > gpurun_out/${P}_bench_notaper.json 2> gpurun_out/${P}_bench_notaper.err || { tail -20 gpurun_out/${P}_bench_notaper.err; exit 1; }
tail -1 gpurun_out/${P}_bench_notaper.json | cut -c1-200
P=${P}p bash tools/gpu/r4_prof3.sh

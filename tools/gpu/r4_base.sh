# round 4 baseline: exact-mode kernel micro-bench, exact bench, in-process
# rocprof kernel table of the exact bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4a}
timeout -k 10 300 python tools/kbench_exact.py > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { tail -20 gpurun_out/${P}_kbench_exact.err; exit 1; }
cat gpurun_out/${P}_kbench_exact.json
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { tail -20 gpurun_out/${P}_bench_exact.err; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 bench.py --exact --in-process --steps 6 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
find gpurun_out/${P}_prof -name "*kernel_stats.csv" | head -3

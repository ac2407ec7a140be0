# kernel table of the exact bench (in-process) + the default bench, both 1 GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4n}
df -h /tmp . | tail -2
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
tail -1 gpurun_out/${P}_bench.json | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 bench.py --exact --in-process --steps 6 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
grep '"metric"' gpurun_out/${P}_prof.log | cut -c1-300

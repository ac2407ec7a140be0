# kernel tables of the default (exact) bench: in-process and worker mode, plus
# the stock-policy reference point
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4w}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_inproc -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/${P}_inproc.log 2>&1 || { tail -20 gpurun_out/${P}_inproc.log; exit 1; }
grep '"metric"' gpurun_out/${P}_inproc.log | cut -c1-200
python tools/rocpd_summary.py $(find gpurun_out/${P}_inproc -name "*.db" | head -1) --iterations --from-last kmeans_assign_top3_grouped 64 --top 30 > gpurun_out/${P}_inproc.md 2>&1
tail -14 gpurun_out/${P}_inproc.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_worker -o run -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/${P}_worker.log 2>&1 || { tail -20 gpurun_out/${P}_worker.log; exit 1; }
grep '"metric"' gpurun_out/${P}_worker.log | cut -c1-200
find gpurun_out/${P}_worker -name "*.db"
timeout -k 10 400 python bench.py --policy stock --steps 1 --warmup 1 > gpurun_out/${P}_stock.json 2> gpurun_out/${P}_stock.err || { tail -20 gpurun_out/${P}_stock.err; exit 1; }
tail -1 gpurun_out/${P}_stock.json | cut -c1-300

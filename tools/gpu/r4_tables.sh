# kernel tables + iteration spans of the default exact bench: in-process and
# worker mode (the driver's configuration)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4t}
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_inproc -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/${P}_inproc.log 2>&1 || { tail -20 gpurun_out/${P}_inproc.log; exit 1; }
grep '"metric"' gpurun_out/${P}_inproc.log | cut -c1-200
DB=$(find /tmp/${P}_inproc -name "*.db" | head -1)
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 7 --top 24 > gpurun_out/${P}_inproc.md 2>&1
head -20 gpurun_out/${P}_inproc.md; tail -9 gpurun_out/${P}_inproc.md
rm -rf /tmp/${P}_inproc
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_worker -o run -- python3 bench.py > gpurun_out/${P}_worker.log 2>&1 || { tail -20 gpurun_out/${P}_worker.log; exit 1; }
grep '"metric"' gpurun_out/${P}_worker.log | cut -c1-200
DB=$(ls -S $(find /tmp/${P}_worker -name "*.db") | head -1)
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 10 --top 24 > gpurun_out/${P}_worker.md 2>&1
tail -12 gpurun_out/${P}_worker.md
rm -rf /tmp/${P}_worker

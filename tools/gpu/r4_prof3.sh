# kernel tables of the default (exact) bench, in-process and worker mode, with
# a host-trace merge around iteration boundaries; the SQLite results are
# summarised on the box and deleted (gpurun copies back <= 64 MiB)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4x}
rm -f /tmp/${P}_trace*.jsonl
HBMR_TRACE=/tmp/${P}_trace.jsonl timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${P}_inproc -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/${P}_inproc.log 2>&1 || { tail -20 gpurun_out/${P}_inproc.log; exit 1; }
grep '"metric"' gpurun_out/${P}_inproc.log | cut -c1-200
DB=$(find /tmp/${P}_inproc -name "*.db" | head -1)
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 6 --top 40 > gpurun_out/${P}_inproc.md 2>&1
python tools/trace_merge.py $DB /tmp/${P}_trace.jsonl --iters 2 > gpurun_out/${P}_merge.txt 2>&1 || true
tail -12 gpurun_out/${P}_inproc.md
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${P}_worker -o run -- python3 bench.py --steps 8 --warmup 3 > gpurun_out/${P}_worker.log 2>&1 || { tail -20 gpurun_out/${P}_worker.log; exit 1; }
grep '"metric"' gpurun_out/${P}_worker.log | cut -c1-200
for DB in $(find /tmp/${P}_worker -name "*.db"); do python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 6 --top 40 >> gpurun_out/${P}_worker.md 2>&1; done
tail -12 gpurun_out/${P}_worker.md
rm -rf /tmp/${P}_inproc /tmp/${P}_worker

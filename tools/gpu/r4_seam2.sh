# in-process exact bench under a kernel trace with the host trace; keeps the
# raw host trace (small) and the merged timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4s2}
rm -f /tmp/${P}_trace*.jsonl
HBMR_TRACE=/tmp/${P}_trace.jsonl timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_inproc -o run -- python3 bench.py --in-process --steps 6 --warmup 3 > gpurun_out/${P}_inproc.log 2>&1 || { tail -20 gpurun_out/${P}_inproc.log; exit 1; }
grep '"metric"' gpurun_out/${P}_inproc.log | cut -c1-200
DB=$(find /tmp/${P}_inproc -name "*.db" | head -1)
python tools/trace_merge.py $DB /tmp/${P}_trace.jsonl --iters 2 > gpurun_out/${P}_merge.txt 2>&1 || true
gzip -c /tmp/${P}_trace.jsonl > gpurun_out/${P}_trace.jsonl.gz
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 5 --top 12 > gpurun_out/${P}_inproc.md 2>&1
tail -8 gpurun_out/${P}_inproc.md
rm -rf /tmp/${P}_inproc

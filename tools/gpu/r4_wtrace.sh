# worker-mode default bench with host traces of every process (main + GPU
# worker) and a kernel trace; merged timeline of the last iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4wt}
rm -rf /tmp/${P}_tr; mkdir -p /tmp/${P}_tr
HBMR_TRACE=/tmp/${P}_tr/t_{pid}.jsonl timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_worker -o run -- python3 bench.py > gpurun_out/${P}_worker.log 2>&1 || { tail -20 gpurun_out/${P}_worker.log; exit 1; }
grep '"metric"' gpurun_out/${P}_worker.log | cut -c1-200
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/${P}_worker.log') if l.startswith('{\"metric')][-1]; print(d['ms_per_step'], d['release_to_finish_ms_per_job'])"
cat /tmp/${P}_tr/*.jsonl > /tmp/${P}_all.jsonl
gzip -c /tmp/${P}_all.jsonl > gpurun_out/${P}_trace.jsonl.gz
DB=$(ls -S $(find /tmp/${P}_worker -name "*.db") | head -1)
python tools/trace_merge.py $DB /tmp/${P}_all.jsonl --iters 4 > gpurun_out/${P}_merge.txt 2>&1 || true
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 10 --top 6 > gpurun_out/${P}_worker.md 2>&1
tail -12 gpurun_out/${P}_worker.md
rm -rf /tmp/${P}_worker

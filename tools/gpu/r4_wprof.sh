# worker-mode default bench under a kernel trace: per-iteration device spans
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4w}
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_worker -o run -- python3 bench.py > gpurun_out/${P}_worker.log 2>&1 || { tail -20 gpurun_out/${P}_worker.log; exit 1; }
grep '"metric"' gpurun_out/${P}_worker.log | cut -c1-200
for DB in $(find /tmp/${P}_worker -name "*.db"); do python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 10 --top 14 >> gpurun_out/${P}_worker.md 2>&1; done
tail -14 gpurun_out/${P}_worker.md
rm -rf /tmp/${P}_worker
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['release_to_finish_ms_per_job'], d['phases_ms'])"

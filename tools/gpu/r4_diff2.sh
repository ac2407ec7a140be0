set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4d2}
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/${P}_kb -o run -- python3 $GRAFT_REPO_ROOT/tools/kbench_delta.py > $GRAFT_REPO_ROOT/gpurun_out/${P}_kb.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/${P}_kb.log; exit 1; }
cd $GRAFT_REPO_ROOT
grep '"splits"' gpurun_out/${P}_kb.log
DB=$(find /tmp/${P}_kb -name "*.db" | head -1)
python tools/rocpd_summary.py $DB --top 8 > gpurun_out/${P}_kb.md 2>&1; head -14 gpurun_out/${P}_kb.md
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_kernels.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['release_to_finish_ms_per_job'])"

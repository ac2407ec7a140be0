# delta-diff kernel rewrite: kmeans kernel tests, then kernel table + bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4d}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_kernels.py tests/test_kmeans_exact.py tests/test_gpu_worker.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${P}_inproc -o run -- python3 bench.py --in-process --steps 6 --warmup 3 > gpurun_out/${P}_inproc.log 2>&1 || { tail -20 gpurun_out/${P}_inproc.log; exit 1; }
grep '"metric"' gpurun_out/${P}_inproc.log | cut -c1-200
DB=$(find /tmp/${P}_inproc -name "*.db" | head -1)
python tools/rocpd_summary.py $DB --iterations --from-last kmeans_update 5 --top 14 > gpurun_out/${P}_inproc.md 2>&1
head -24 gpurun_out/${P}_inproc.md | tail -18; tail -6 gpurun_out/${P}_inproc.md
rm -rf /tmp/${P}_inproc
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench$i.json 2> gpurun_out/${P}_bench$i.err || { tail -20 gpurun_out/${P}_bench$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_bench$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['release_to_finish_ms_per_job'])"
done

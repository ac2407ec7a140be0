# final tree: every GPU test, smoke, default bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4fd}
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || { tail -20 gpurun_out/${P}_smoke.txt; exit 1; }
echo smoke ok
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench$i.json 2> gpurun_out/${P}_bench$i.err || { tail -20 gpurun_out/${P}_bench$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_bench$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['release_to_finish_ms_per_job'])"
done

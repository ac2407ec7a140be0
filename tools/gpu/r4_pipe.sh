# epilogue-pipelined top-3 kernel: exact tests with it, then same-box A/B
# (HBMR_EXACT_PIPE=1 vs 0) of the kernel bench and the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4pp}
HBMR_EXACT_PIPE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
for v in 1 0; do
HBMR_EXACT_PIPE=$v timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench$v.json 2> gpurun_out/${P}_kbench$v.err || { tail -20 gpurun_out/${P}_kbench$v.err; exit 1; }
echo "pipe=$v"; cut -c1-400 gpurun_out/${P}_kbench$v.json
done
for i in 1 2; do
for v in 1 0; do
HBMR_EXACT_PIPE=$v timeout -k 10 300 python bench.py > gpurun_out/${P}_b${v}_$i.json 2> gpurun_out/${P}_b${v}_$i.err || { tail -20 gpurun_out/${P}_b${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_b${v}_$i.json').read().strip().splitlines()[-1]); print('pipe=$v', d['ms_per_step'], d.get('final_shift'))"
done
done

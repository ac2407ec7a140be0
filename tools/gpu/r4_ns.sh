# fused top-3 kernel ring depth A/B: HBMR_EXACT_NS=6 vs 4 on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4ns}
HBMR_EXACT_NS=6 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
for v in 6 4 6 4; do
HBMR_EXACT_NS=$v timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 --reps 8 > gpurun_out/${P}_kb$v.json 2> gpurun_out/${P}_kb$v.err || { tail -20 gpurun_out/${P}_kb$v.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_kb$v.json').read().strip().splitlines()[-1]); print('ns=$v exact_batch_ms', d['exact_batch_ms'])"
done
for i in 1 2; do
for v in 6 4; do
HBMR_EXACT_NS=$v timeout -k 10 300 python bench.py > gpurun_out/${P}_b${v}_$i.json 2> gpurun_out/${P}_b${v}_$i.err || { tail -20 gpurun_out/${P}_b${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_b${v}_$i.json').read().strip().splitlines()[-1]); print('ns=$v', d['ms_per_step'], d.get('final_shift'))"
done
done

# stock vs hybrid scheduling on the current tree, and the default bench at
# 10 and 20 timed jobs (the first timed job's launch is not pre-staged)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4s}
timeout -k 10 300 python bench.py --policy stock --steps 1 --warmup 1 > gpurun_out/${P}_stock.json 2> gpurun_out/${P}_stock.err || { tail -20 gpurun_out/${P}_stock.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_stock.json').read().strip().splitlines()[-1]); print('stock', d['ms_per_step'])"
timeout -k 10 300 python bench.py > gpurun_out/${P}_hybrid10.json 2> gpurun_out/${P}_hybrid10.err || { tail -20 gpurun_out/${P}_hybrid10.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_hybrid10.json').read().strip().splitlines()[-1]); print('hybrid 10 jobs', d['ms_per_step'], d['release_to_finish_ms_per_job'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_hybrid20.json 2> gpurun_out/${P}_hybrid20.err || { tail -20 gpurun_out/${P}_hybrid20.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_hybrid20.json').read().strip().splitlines()[-1]); print('hybrid 20 jobs', d['ms_per_step'], d['release_to_finish_ms_per_job'])"

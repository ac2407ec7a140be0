# hardware queues per process: 8 vs HIP's default 4, default bench, one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4q}
for i in 1 2; do
for v in 8 4; do
GPU_MAX_HW_QUEUES=$v timeout -k 10 300 python bench.py > gpurun_out/${P}_h${v}_$i.json 2> gpurun_out/${P}_h${v}_$i.err || { tail -20 gpurun_out/${P}_h${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_h${v}_$i.json').read().strip().splitlines()[-1]); print('hwq=$v', d['ms_per_step'], d['release_to_finish_ms_per_job'][:4])"
done
done

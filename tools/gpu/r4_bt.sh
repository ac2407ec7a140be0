# staged batch target A/B after the seam fixes: 16 (default) vs 32 vs 24
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for v in 32 16 24; do
timeout -k 10 300 python bench.py -D hbmr.gpu.batch.target=$v > gpurun_out/r4bt_${v}_$i.json 2> gpurun_out/r4bt_${v}_$i.err || { tail -20 gpurun_out/r4bt_${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4bt_${v}_$i.json').read().strip().splitlines()[-1]); print('target=$v', d['ms_per_step'])"
done
done

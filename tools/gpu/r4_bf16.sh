set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python bench.py --no-exact > gpurun_out/r4bf_$i.json 2> gpurun_out/r4bf_$i.err || { tail -20 gpurun_out/r4bf_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4bf_$i.json').read().strip().splitlines()[-1]); print('bf16', d['ms_per_step'], d['dtype'], d['release_to_finish_ms_per_job'])"
done

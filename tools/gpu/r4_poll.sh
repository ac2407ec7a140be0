# completer polling A/B: worker-mode trace with polling (default), then the
# default bench with polling and with blocking synchronize, twice each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=r4pt bash tools/gpu/r4_wtrace.sh || exit 1
for i in 1 2; do
for v in 100 0; do
timeout -k 10 300 python bench.py -D hbmr.gpu.completion.poll.us=$v > gpurun_out/r4p_b${v}_$i.json 2> gpurun_out/r4p_b${v}_$i.err || { tail -20 gpurun_out/r4p_b${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4p_b${v}_$i.json').read().strip().splitlines()[-1]); print('poll $v', d['ms_per_step'], d['release_to_finish_ms_per_job'])"
done
done

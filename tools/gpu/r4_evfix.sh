# reduce marker events A/B: seam trace, then the default (worker-mode) bench twice
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4e}
P=${P}s bash tools/gpu/r4_seam2.sh || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench$i.json 2> gpurun_out/${P}_bench$i.err || { tail -20 gpurun_out/${P}_bench$i.err; exit 1; }
tail -1 gpurun_out/${P}_bench$i.json | cut -c1-400
done

# A/B on one box: iteration jobs prefetched (default) vs not
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --prefetch > gpurun_out/ab_pre_$i.log 2>&1 && grep '^{' gpurun_out/ab_pre_$i.log | tail -1 | cut -c150-200 || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_nopre_$i.log 2>&1 && grep '^{' gpurun_out/ab_nopre_$i.log | tail -1 | cut -c150-200 || exit 1
done

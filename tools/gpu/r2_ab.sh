# A/B of the 1-GPU bench on one box: base worktree vs this tree, alternating
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  (cd abtest/base && timeout -k 10 200 python bench.py --steps 20 --warmup 5 > ../../gpurun_out/ab_base_$i.log 2>&1) && grep '^{' gpurun_out/ab_base_$i.log | tail -1 | cut -c150-200 || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/ab_head_$i.log 2>&1 && grep '^{' gpurun_out/ab_head_$i.log | tail -1 | cut -c150-200 || exit 1
done

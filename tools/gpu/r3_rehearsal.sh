# round 3: CPU-only multi-rank rehearsal on the GPU box's host (simulated GPU slots,
# 0.24 ms device time per split as measured on the MI355X), 1/2/4/8 ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3g}
echo "nproc $(nproc)"
for N in 1 2 4 8; do
  HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= timeout -k 10 200 python bench.py --gpus $N --simulate-ms 0.24 --steps 20 --warmup 3 "$@" > gpurun_out/${P}_n$N.json 2> gpurun_out/${P}_n$N.err || { echo "N=$N failed"; tail -5 gpurun_out/${P}_n$N.err; exit 1; }
  tail -1 gpurun_out/${P}_n$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N', d['ms_per_step'], d['phases_ms'])"
done

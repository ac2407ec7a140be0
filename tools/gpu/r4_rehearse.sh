# 1/2/4/8-rank CPU rehearsal on the box's host (simulated 0.24 ms/split GPU
# slots, no device use): JobTracker in rank 0 vs in a process of its own
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4r}
echo "nproc $(nproc)"
for JTP in false true; do
for N in 1 2 4 8; do
  HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= timeout -k 10 200 python bench.py --gpus $N --simulate-ms 0.24 --steps 30 --warmup 3 -D hbmr.jobtracker.process=$JTP > gpurun_out/${P}_${JTP}_n$N.json 2> gpurun_out/${P}_${JTP}_n$N.err || { echo "N=$N failed"; tail -5 gpurun_out/${P}_${JTP}_n$N.err; exit 1; }
  tail -1 gpurun_out/${P}_${JTP}_n$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('jtproc=$JTP N=$N', d['ms_per_step'], 'rank0', d['rank0_cpu_ms_per_step'], 'jt', d.get('jobtracker_cpu_ms_per_step'))"
done
done

# 1/2/4/8-rank CPU rehearsal of the headline job on the box host (simulated
# GPU slots, gloo): ms/job, rank-0 and JobTracker-process CPU per job
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r6r}
: > gpurun_out/${P}_rehearsal.jsonl
for n in ${NS:-1 2 4 8}; do
  for rep in ${REPS:-1 2}; do
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n * 10 + rep)) bench.py --gpus $n --simulate-ms 0.26 --steps 30 --warmup 5 -D hbmr.jobtracker.process=true ${EXTRA:-} > gpurun_out/${P}_n${n}_${rep}.json 2> gpurun_out/${P}_n${n}_${rep}.err || { tail -5 gpurun_out/${P}_n${n}_${rep}.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/${P}_n${n}_${rep}.json').read().strip().splitlines()[-1])
r={'n':$n,'rep':$rep,**{k:d.get(k) for k in ('ms_per_step','rank0_cpu_ms_per_step','jobtracker_cpu_ms_per_step')}}
print(json.dumps(r)); open('gpurun_out/${P}_rehearsal.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

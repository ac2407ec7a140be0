# JobTracker RPC trace + per-method stats of the N-rank CPU rehearsal (simulated GPU slots)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${P:-r5t}
n=${N:-8}
mkdir -p gpurun_out/$P
HBMR_RPC_TRACE=$PWD/gpurun_out/$P/tr HBMR_SAMPLE_PROF=$PWD/gpurun_out/$P/s timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus $n --simulate-ms 0.26 --steps ${STEPS:-30} --warmup 5 -D hbmr.jobtracker.process=true $EXTRA > gpurun_out/$P/n${n}.json 2> gpurun_out/$P/n${n}.err || { tail -5 gpurun_out/$P/n${n}.err; exit 1; }
find gpurun_out/$P -size 0 -delete
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29556 bench.py --gpus $n --simulate-ms 0.26 --steps ${STEPS:-30} --warmup 5 -D hbmr.jobtracker.process=true $EXTRA > gpurun_out/$P/plain_n${n}.json 2> gpurun_out/$P/plain_n${n}.err || { tail -5 gpurun_out/$P/plain_n${n}.err; exit 1; }
python3 -c "
import json,sys
for f in ['n$n','plain_n$n']:
    d=json.loads(open('gpurun_out/$P/'+f+'.json').read().strip().splitlines()[-1])
    print(f, d['ms_per_step'], d.get('jobtracker_cpu_ms_per_step'), d.get('rank0_cpu_ms_per_step'))
"

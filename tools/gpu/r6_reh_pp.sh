#!/bin/bash
# 8-rank CPU rehearsal with the JobTracker's per-method CPU accounting
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
HBMR_PHASE_PROF=$PWD/gpurun_out/r6pp timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29581 bench.py --gpus 8 --simulate-ms 0.26 --steps 100 --warmup 5 -D hbmr.jobtracker.process=true > gpurun_out/r6pp_run.json 2> gpurun_out/r6pp_run.err || { tail -5 gpurun_out/r6pp_run.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/r6pp_run.json').read().strip().splitlines()[-1]);print(d['ms_per_step'],d['jobtracker_cpu_ms_per_step'])"
cat gpurun_out/r6pp_*.txt

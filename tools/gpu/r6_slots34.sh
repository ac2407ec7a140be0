#!/bin/bash
# bench line: 2 (default) vs 3 vs 4 GPU map slots per GPU, interleaved
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_slots34.jsonl
for rep in 1 2; do
  for n in 2 3 4; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --gpu-slots $n > gpurun_out/r6_s34.json 2> gpurun_out/r6_s34.err || { tail -5 gpurun_out/r6_s34.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/r6_s34.json').read().strip().splitlines()[-1])
r={'gpu_slots':$n,'rep':$rep,'ms_per_step':d['ms_per_step'],'map_device_ms_per_job':d.get('map_device_ms_per_job')}
print(json.dumps(r)); open('gpurun_out/r6_slots34.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

#!/bin/bash
# bench line: GPU map slots per GPU and batch target A/B (interleaved)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_slots_ab.jsonl
for rep in 1 2; do
  for cfg in "--gpu-slots 2" "--gpu-slots 1" "--gpu-slots 2 -D hbmr.gpu.batch.target=32" "--gpu-slots 1 -D hbmr.gpu.batch.target=32"; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 $cfg > gpurun_out/r6_sab.json 2> gpurun_out/r6_sab.err || { tail -5 gpurun_out/r6_sab.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/r6_sab.json').read().strip().splitlines()[-1])
r={'cfg':'$cfg','rep':$rep,'ms_per_step':d['ms_per_step'],'map_device_ms_per_job':d.get('map_device_ms_per_job')}
print(json.dumps(r)); open('gpurun_out/r6_slots_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

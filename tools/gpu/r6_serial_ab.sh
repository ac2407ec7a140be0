#!/bin/bash
# bench line: GPU slots overlapping kernels (default) vs serialised on the device
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_serial_ab.jsonl
for rep in 1 2 3; do
  for mode in false true; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 -D hbmr.gpu.slots.serialize=$mode > gpurun_out/r6_ser.json 2> gpurun_out/r6_ser.err || { tail -5 gpurun_out/r6_ser.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/r6_ser.json').read().strip().splitlines()[-1])
r={'serialize':'$mode','rep':$rep,'ms_per_step':d['ms_per_step'],'map_device_ms_per_job':d.get('map_device_ms_per_job')}
print(json.dumps(r)); open('gpurun_out/r6_serial_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

#!/bin/bash
# exact batch time vs the refine (q2/q3) persistent grid size
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_refine_grid.jsonl
for g in 2048 768 1024 1536 3072 2048; do
  HBMR_REFINE_GRID=$g timeout -k 10 120 python3 -u tools/kbench_v3.py --modes v3 --reps 11 > gpurun_out/r6_rg.txt 2>&1 || { tail -5 gpurun_out/r6_rg.txt; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r6_rg.txt') if l.startswith('{')][-1]
d['grid']=$g; print(json.dumps(d)); open('gpurun_out/r6_refine_grid.jsonl','a').write(json.dumps(d)+'\n')"
done

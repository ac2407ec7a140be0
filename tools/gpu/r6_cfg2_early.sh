#!/bin/bash
# config 2: the reduce launched with the maps (slow-start 0, default) vs after the first report
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_cfg2_early.jsonl
for rep in 1 2 3; do
  for early in true false; do
    timeout -k 10 240 python -u tools/bench_configs.py kmeans-pipes --steps 20 -D hbmr.kmeans.pipes.reduce.early=$early > gpurun_out/r6_c2e.json 2> gpurun_out/r6_c2e.err || { tail -5 gpurun_out/r6_c2e.err; exit 1; }
    python3 -c "
import json,statistics
d=json.loads(open('gpurun_out/r6_c2e.json').read().strip().splitlines()[-1])
it=d['pipes_iteration_s']
r={'reduce_early':'$early','rep':$rep,'median_ms':round(statistics.median(it)*1e3,2),'min_ms':round(min(it)*1e3,2)}
print(json.dumps(r)); open('gpurun_out/r6_cfg2_early.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

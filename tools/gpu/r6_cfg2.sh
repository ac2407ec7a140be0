#!/bin/bash
# BASELINE config 2 (Pipes K-Means 1M x 128, k=64, 8 GPU maps): per-iteration
# medians over fresh processes, defaults
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_cfg2.jsonl
for rep in 1 2 3 4 5; do
  timeout -k 10 240 python -u tools/bench_configs.py kmeans-pipes --steps 20 > gpurun_out/r6_cfg2_run.json 2> gpurun_out/r6_cfg2_err.log || exit $?
  python3 -c "
import json,statistics
d=json.loads(open('gpurun_out/r6_cfg2_run.json').read().strip().splitlines()[-1])
it=d['pipes_iteration_s']
r={'rep':$rep,'median_ms':round(statistics.median(it)*1e3,2),'min_ms':round(min(it)*1e3,2),'splitjob_median_ms':round(statistics.median(d.get('splitjob_iteration_ms') or [0]),2)}
print(json.dumps(r)); open('gpurun_out/r6_cfg2.jsonl','a').write(json.dumps(r)+'\n')"
done

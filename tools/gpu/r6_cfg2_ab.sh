#!/bin/bash
# BASELINE config 2 (Pipes K-Means, 8 GPU maps per iteration): per-batch
# reports of bulk-launched per-attempt GPU maps on/off, fresh processes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/r6_cfg2_ab.jsonl
for rep in 1 2 3; do
  for mode in true false; do
    timeout -k 10 240 python -u tools/bench_configs.py kmeans-pipes --steps 20 \
      -D hbmr.tracker.batch.reports=$mode > gpurun_out/r6_cfg2_$mode_$rep.json 2> gpurun_out/r6_cfg2_err.log || exit $?
    python3 -c "
import json,statistics
d=json.loads(open('gpurun_out/r6_cfg2_$mode_$rep.json').read().strip().splitlines()[-1])
it=d['pipes_iteration_s']
r={'batch_reports':'$mode','rep':$rep,'median_ms':round(statistics.median(it)*1e3,2),'min_ms':round(min(it)*1e3,2),'splitjob_ms':d.get('splitjob_iteration_ms')}
print(json.dumps(r)); open('gpurun_out/r6_cfg2_ab.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

#!/bin/bash
# config 2: bulk launch + prelaunch (default) vs prelaunch off vs per-task launches (round-6 start)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmeans_pipes.py tests/test_pipes_prelaunch.py -m "gpu or not gpu" > gpurun_out/r6_cfg2_pre_tests.log 2>&1 || { tail -30 gpurun_out/r6_cfg2_pre_tests.log; exit 1; }
tail -1 gpurun_out/r6_cfg2_pre_tests.log
: > gpurun_out/r6_cfg2_pre.jsonl
for rep in 1 2 3; do
  for cfg in "default" "-D hbmr.pipes.gpu.prelaunch=false" "-D hbmr.scheduler.gpu.bulk.classic=false"; do
    args=""; [ "$cfg" != "default" ] && args="$cfg"
    timeout -k 10 240 python -u tools/bench_configs.py kmeans-pipes --steps 20 $args > gpurun_out/r6_c2p.json 2> gpurun_out/r6_c2p.err || { tail -5 gpurun_out/r6_c2p.err; exit 1; }
    python3 -c "
import json,statistics
d=json.loads(open('gpurun_out/r6_c2p.json').read().strip().splitlines()[-1])
it=d['pipes_iteration_s']
r={'cfg':'$cfg','rep':$rep,'median_ms':round(statistics.median(it)*1e3,2),'min_ms':round(min(it)*1e3,2)}
print(json.dumps(r)); open('gpurun_out/r6_cfg2_pre.jsonl','a').write(json.dumps(r)+'\n')"
  done
done

#!/bin/bash
# final round-6 pass: GPU tests, config 2 medians (3 fresh processes), bench line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6_gpu_tests.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc"; tail -2 gpurun_out/r6_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
: > gpurun_out/r6_cfg2_final.jsonl
for rep in 1 2 3; do
  timeout -k 10 240 python -u tools/bench_configs.py kmeans-pipes --steps 20 > gpurun_out/r6_c2f.json 2> gpurun_out/r6_c2f.err || exit $?
  python3 -c "
import json,statistics
d=json.loads(open('gpurun_out/r6_c2f.json').read().strip().splitlines()[-1])
it=d['pipes_iteration_s']
r={'rep':$rep,'median_ms':round(statistics.median(it)*1e3,2),'min_ms':round(min(it)*1e3,2)}
print(json.dumps(r)); open('gpurun_out/r6_cfg2_final.jsonl','a').write(json.dumps(r)+'\n')"
done
timeout -k 10 300 python -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
rc2=$?
echo "BENCH_EXIT $rc2"
cut -c1-400 gpurun_out/r6_bench.json
exit $rc2

#!/bin/bash
# Config 2 (K-Means 1M x 128, k=64, Pipes GPU binary) in 5 fresh processes, and
# config 1 (WordCount, LocalJobRunner) serial vs 8 warm map processes.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r6cfg}
: > gpurun_out/${P}_summary.txt
for rep in 1 2 3 4 5; do
  timeout -k 10 240 python3 -u tools/bench_configs.py kmeans-pipes --steps 20 \
    > gpurun_out/${P}_c2_${rep}.json 2> gpurun_out/${P}_c2_${rep}.err || { tail -20 gpurun_out/${P}_c2_${rep}.err; exit 1; }
  python3 -c "import json,statistics as s;d=json.load(open('gpurun_out/${P}_c2_${rep}.json'));t=d['pipes_iteration_s'][3:];print('config2 rep',$rep,'median_ms',round(1e3*s.median(t),2),'min_ms',round(1e3*min(t),2))" | tee -a gpurun_out/${P}_summary.txt
done
for pr in 1 8; do
  timeout -k 10 240 python3 -u tools/bench_configs.py wordcount --mb 64 --steps 5 --procs $pr \
    > gpurun_out/${P}_c1_$pr.json 2> gpurun_out/${P}_c1_$pr.err || { tail -20 gpurun_out/${P}_c1_$pr.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${P}_c1_$pr.json'));print('config1 procs',$pr,d['job_seconds'],d['mb_per_s'])" | tee -a gpurun_out/${P}_summary.txt
done

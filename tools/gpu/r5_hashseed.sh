# Config 2 per fresh process with fixed hash seeds: is the run-to-run spread
# an ordering effect?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5hs}
: > gpurun_out/${P}_summary.txt
for rep in 1 2 3; do
  for seed in 0 1; do
    PYTHONHASHSEED=$seed timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 15 > gpurun_out/${P}_${seed}_${rep}.json 2> gpurun_out/${P}_${seed}_${rep}.err || { tail -20 gpurun_out/${P}_${seed}_${rep}.err; exit 1; }
    python3 -c "import json,statistics as s;d=json.load(open('gpurun_out/${P}_${seed}_${rep}.json'));t=d['pipes_iteration_s'][3:];print('seed',$seed,'rep',$rep,'median_ms',round(1e3*s.median(t),2))" | tee -a gpurun_out/${P}_summary.txt
  done
done

# Config 2 over hbmr.pipes.gpu.queue.depth (map threads per GPU Pipes child), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5dp}
: > gpurun_out/${P}_summary.txt
for rep in ${REPS:-1 2}; do
  for dpt in ${DEPTHS:-2 4 8}; do
    timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 20 -D hbmr.pipes.gpu.queue.depth=$dpt > gpurun_out/${P}_${dpt}_${rep}.json 2> gpurun_out/${P}_${dpt}_${rep}.err || { tail -20 gpurun_out/${P}_${dpt}_${rep}.err; exit 1; }
    python3 -c "import json,statistics as s;d=json.load(open('gpurun_out/${P}_${dpt}_${rep}.json'));t=d['pipes_iteration_s'][3:];print('depth',$dpt,'rep',$rep,'median_ms',round(1e3*s.median(t),2),'min_ms',round(1e3*min(t),2))" | tee -a gpurun_out/${P}_summary.txt
  done
done

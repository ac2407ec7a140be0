# Config 2 A/B on one box: Pipes byte paths on (raw) vs off (obj), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5ab}
for m in raw obj raw obj; do
  if [ $m = raw ]; then R=1; else R=0; fi
  HBMR_PIPES_RAW=$R timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 25 > gpurun_out/${P}_${m}.json 2> gpurun_out/${P}_${m}.err || { tail -20 gpurun_out/${P}_${m}.err; exit 1; }
  python3 -c "import json,statistics as s;d=json.load(open('gpurun_out/${P}_${m}.json'));t=d['pipes_iteration_s'][3:];print('$m', 'median_ms', round(1e3*s.median(t),2), 'min_ms', round(1e3*min(t),2))" | tee -a gpurun_out/${P}_summary.txt
done

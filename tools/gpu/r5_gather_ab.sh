# gather variants A/B at 100 GB: 16-B pieces with 4 / 8 records in flight per lane, plain / NT stores
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P=${P:-r5ga}
for mode in def u8 nt u8nt def; do
  if [ $mode = def ]; then unset HBMR_GATHER; else export HBMR_GATHER=$mode; fi
  timeout -k 10 600 python3 tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/${P}_$mode.json 2> gpurun_out/${P}_$mode.err || { tail -5 gpurun_out/${P}_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${P}_$mode.json').read().strip().splitlines()[-1]);print('$mode', d['seconds_per_sort'], d['gb_per_s'], d['validated'])"
done

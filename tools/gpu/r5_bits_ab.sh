# TeraSort radix window 48 (6 passes) vs 40 bits (5 passes, ties on the 40-bit prefix fixed in place)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P=${P:-r5bits}
for b in 48 40 48 40; do
  HBMR_TERA_SORT_BITS=$b timeout -k 10 600 python3 tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/${P}_$b.json 2> gpurun_out/${P}_$b.err || { tail -5 gpurun_out/${P}_$b.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${P}_$b.json').read().strip().splitlines()[-1]);print('$b', d['seconds_per_sort'], d['gb_per_s'], d['validated'])"
done

# round 3 (late): TeraSort 100 GB record-gather A/B (HBMR_GATHER = default,
# u8, nt, u8nt) and the 40-bit radix window, one box, back to back
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3g}
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_terasort.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
for V in def u8 nt u8nt def bits40; do
  if [ $V = bits40 ]; then E="HBMR_TERA_SORT_BITS=40"; elif [ $V = def ]; then E="HBMR_GATHER="; else E="HBMR_GATHER=$V"; fi
  timeout -k 10 300 env $E python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_$V.json 2> gpurun_out/${P}_$V.err || { tail -20 gpurun_out/${P}_$V.err; exit 1; }
  echo "$V $(tail -1 gpurun_out/${P}_$V.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["seconds_per_sort"], d["gb_per_s"], d["validated"])')"
done

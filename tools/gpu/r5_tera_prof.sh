# TeraSort kernel stats (rocprofv3) for the default and v1 map/gather kernels at 20 GB,
# and (OUT=1) an output-committed sort to the box's overlay root sized to its free space
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5tp}
for mode in default v1; do
  if [ $mode = default ]; then unset HBMR_GATHER HBMR_TERA_PART; else export HBMR_GATHER=w1 HBMR_TERA_PART=v1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_$mode -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 2 > gpurun_out/${P}_$mode.log 2>&1 || { tail -5 gpurun_out/${P}_$mode.log; exit 1; }
  tail -1 gpurun_out/${P}_$mode.log | cut -c1-200
  f=$(find gpurun_out/${P}_$mode -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:10]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d}  {r["Name"][:90]}')
PY
done
unset HBMR_GATHER HBMR_TERA_PART
if [ "${OUT:-0}" = 1 ]; then
  D=$GRAFT_REPO_ROOT/tera-out-durable
  FREE=$(python3 -c "import shutil;print(shutil.disk_usage('$GRAFT_REPO_ROOT').free)")
  ROWS=$(python3 -c "print(min(1000000000, int($FREE/100/1.3)//10000000*10000000))")
  echo "durable: $(stat -f -c %T $GRAFT_REPO_ROOT) free=$FREE rows=$ROWS"
  timeout -k 10 900 python3 tools/bench_terasort.py --rows $ROWS --steps 1 --warmup 1 --output $D > gpurun_out/${P}_durable.json 2> gpurun_out/${P}_durable.err || { tail -5 gpurun_out/${P}_durable.err; rm -rf $D; exit 1; }
  rm -rf $D
  tail -c 700 gpurun_out/${P}_durable.json
fi

# 1-GPU bench (plain) + rocprofv3 kernel stats of the bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5bp}
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -5 gpurun_out/${P}_bench.err; exit 1; }
python3 -c "
import json;d=json.loads(open('gpurun_out/${P}_bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['map_device_ms_per_job'], json.dumps(d['cost_model']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_prof -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -5 gpurun_out/${P}_prof.log; exit 1; }
f=$(find gpurun_out/${P}_prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} {100*float(r["TotalDurationNs"])/tot:5.1f}%  {r["Name"][:80]}')
PY

# TeraSort: gather-piece test + job tests, 100 GB in HBM (16-B-piece gather vs word-per-lane),
# then (OUT=1) the output-committed sort to a non-tmpfs path with fsync when one has the space
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5ts}
df -h /tmp $GRAFT_REPO_ROOT $HOME /dev/shm > gpurun_out/${P}_df.txt 2>&1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_terasort.py -m gpu -k "gather or terasort_job or commits_output or many_partitions or partition or radix" > gpurun_out/${P}_tests.log 2>&1 || { tail -20 gpurun_out/${P}_tests.log; exit 1; }
tail -1 gpurun_out/${P}_tests.log
for mode in default v1 default; do
  if [ $mode = default ]; then unset HBMR_GATHER HBMR_TERA_PART; else export HBMR_GATHER=w1 HBMR_TERA_PART=v1; fi
  timeout -k 10 600 python3 tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/${P}_100g_$mode.json 2> gpurun_out/${P}_100g_$mode.err || { tail -5 gpurun_out/${P}_100g_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${P}_100g_$mode.json').read().strip().splitlines()[-1]);print('$mode', d['seconds_per_sort'], d['gb_per_s'], d['validated'])"
done
unset HBMR_GATHER
if [ "${OUT:-0}" = 1 ]; then
  D=$(python3 - <<'PY'
import os, shutil, subprocess
for d in [os.environ.get("GRAFT_REPO_ROOT", "."), os.environ.get("HOME", "/"), "/tmp", "/var/tmp"]:
    try:
        fs = subprocess.run(["stat", "-f", "-c", "%T", d], capture_output=True, text=True).stdout.strip()
        free = shutil.disk_usage(d).free
    except Exception:
        continue
    if fs not in ("tmpfs", "ramfs") and free > 130e9:
        print(os.path.join(d, "tera-out-durable")); break
PY
)
  echo "durable dir: ${D:-none}"
  if [ -n "$D" ]; then
    timeout -k 10 900 python3 tools/bench_terasort.py --rows 1000000000 --steps 1 --warmup 1 --output $D > gpurun_out/${P}_100g_durable.json 2> gpurun_out/${P}_100g_durable.err || { tail -5 gpurun_out/${P}_100g_durable.err; rm -rf $D; exit 1; }
    stat -f -c "%T" $(dirname $D) > gpurun_out/${P}_durable_fs.txt
    rm -rf $D
    tail -c 600 gpurun_out/${P}_100g_durable.json
  fi
fi

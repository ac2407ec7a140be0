# round 3: same-box A/B of the tracker news path: report RPC + deferred map
# reports (default) vs wakeup + immediate reports (round-3 start), 3 runs each,
# interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3t}
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_new_$i.json 2> gpurun_out/${P}_new_$i.err || { grep -v amdgpu.ids gpurun_out/${P}_new_$i.err | tail -20; exit 1; }
  tail -1 gpurun_out/${P}_new_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('new', d['ms_per_step'], d['rank0_cpu_ms_per_step'])"
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 -D hbmr.tracker.report.news=false -D hbmr.tracker.defer.map.reports=false > gpurun_out/${P}_old_$i.json 2> gpurun_out/${P}_old_$i.err || { grep -v amdgpu.ids gpurun_out/${P}_old_$i.err | tail -20; exit 1; }
  tail -1 gpurun_out/${P}_old_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('old', d['ms_per_step'], d['rank0_cpu_ms_per_step'])"
done

# round 3: file-backed bench with splits sized by the map count (128 x 419 MB)
# and the exact bench after the refine counter fix
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3w}
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --exact > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_bench_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['ms_per_step'], d['phases_ms'])"
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km100m > gpurun_out/${P}_write100.txt 2>&1 || { tail -5 gpurun_out/${P}_write100.txt; exit 1; }
tail -1 gpurun_out/${P}_write100.txt
HBMR_STACKDUMP_S=30 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --verbose --input /tmp/km100m > gpurun_out/${P}_bench_file100.json 2> gpurun_out/${P}_bench_file100.err
rc=$?
grep -A6 "bench:\|jt-watch\|worker-watch" gpurun_out/${P}_bench_file100.err | grep -v "^  File\|^Thread" | head -30
echo "file100 rc=$rc"
[ $rc -eq 0 ] && tail -1 gpurun_out/${P}_bench_file100.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file100', d['ms_per_step'], d['warmup_seconds'], d['cpu_maps'], d['config']['map_tasks_per_job'], d['maps_launched'], d['cost_model'])"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { grep -v amdgpu.ids gpurun_out/${P}_bench.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['rank0_cpu_ms_per_step'])"

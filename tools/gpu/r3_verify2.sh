# round 3: verification of the current tree (report RPC, deferred map reports,
# TeraSort v4 default, exact-mode fix, prestage queue fix): GPU tests, the
# default and exact bench, and the file-backed bench at 100M points
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3r}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${P}_gpu_tests.txt
timeout -k 10 150 python tools/kbench_exact.py > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_kbench_exact.err | tail -20; exit 1; }
cat gpurun_out/${P}_kbench_exact.json
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { grep -v amdgpu.ids gpurun_out/${P}_bench.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['rank0_cpu_ms_per_step'], d['phases_ms'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --exact > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_bench_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['ms_per_step'], d['phases_ms'])"
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km100m > gpurun_out/${P}_write100.txt 2>&1 || { tail -5 gpurun_out/${P}_write100.txt; exit 1; }
tail -1 gpurun_out/${P}_write100.txt
HBMR_STACKDUMP_S=30 timeout -k 10 200 python bench.py --steps 10 --warmup 3 --verbose --input /tmp/km100m > gpurun_out/${P}_bench_file100.json 2> gpurun_out/${P}_bench_file100.err
rc=$?
grep -A6 "bench:\|jt-watch\|worker-watch" gpurun_out/${P}_bench_file100.err | grep -v "^  File\|^Thread" | head -30
echo "file100 rc=$rc"
[ $rc -eq 0 ] && tail -1 gpurun_out/${P}_bench_file100.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file100', d['ms_per_step'], d['warmup_seconds'], d['cpu_maps'], d['config']['map_tasks_per_job'], d['cost_model'])"
exit $rc

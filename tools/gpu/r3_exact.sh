# round 3: exact mode with the certification bound on the actual rounding
# errors: its GPU tests, the kernel micro-benchmark and the exact bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3p}
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py > gpurun_out/${P}_exact_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_exact_tests.txt; exit 1; }
grep -E "agreement|passed|failed" gpurun_out/${P}_exact_tests.txt
timeout -k 10 150 python tools/kbench_exact.py > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_kbench_exact.err | tail -20; exit 1; }
cat gpurun_out/${P}_kbench_exact.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --exact > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_bench_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['dtype'], d['ms_per_step'], d['phases_ms'])"
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km20m --points 20000000 > gpurun_out/${P}_write20.txt 2>&1 || { tail -5 gpurun_out/${P}_write20.txt; exit 1; }
HBMR_STACKDUMP_S=20 timeout -k 10 75 python bench.py --steps 5 --warmup 2 --verbose --input /tmp/km20m --points 20000000 > gpurun_out/${P}_bench_file20.json 2> gpurun_out/${P}_bench_file20.err
rc=$?
grep -A6 "bench:\|jt-watch\|worker-watch" gpurun_out/${P}_bench_file20.err | grep -v "^  File\|^Thread" | head -40
echo "file20 rc=$rc"
exit $rc

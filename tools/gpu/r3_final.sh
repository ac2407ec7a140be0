# round 3 (late session): verify the restored tree on the GPU —
# GPU tests, smoke(), the default bench and the exact-mode bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3z}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || { tail -20 gpurun_out/${P}_smoke.txt; exit 1; }
tail -1 gpurun_out/${P}_smoke.txt
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { grep -v amdgpu.ids gpurun_out/${P}_bench.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'])"
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_exact.json 2> gpurun_out/${P}_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['ms_per_step'])"
# exact-mode kernels: refine v1 (HBMR_REFINE=1) vs v2 (default)
timeout -k 10 240 env HBMR_REFINE=1 python tools/kbench_exact.py > gpurun_out/${P}_kx_v1.json 2> gpurun_out/${P}_kx_v1.err || { tail -20 gpurun_out/${P}_kx_v1.err; exit 1; }
timeout -k 10 240 python tools/kbench_exact.py > gpurun_out/${P}_kx_v2.json 2> gpurun_out/${P}_kx_v2.err || { tail -20 gpurun_out/${P}_kx_v2.err; exit 1; }
grep -h refine gpurun_out/${P}_kx_v1.json gpurun_out/${P}_kx_v2.json | cut -c1-400
# TeraSort 100 GB kernel table
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_tprof -o run -- python3 tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 2 > gpurun_out/${P}_tprof.log 2>&1 || { tail -20 gpurun_out/${P}_tprof.log; exit 1; }
tail -1 gpurun_out/${P}_tprof.log | cut -c1-300
for db in $(find gpurun_out/${P}_tprof -name "*.db"); do
  python tools/rocpd_summary.py $db --top 24 > gpurun_out/${P}_tera100_summary.md || true
done

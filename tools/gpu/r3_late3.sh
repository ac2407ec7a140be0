# round 3 (late): batched exact assign; whole-tree GPU tests, smoke, bench,
# exact bench, TeraSort 100 GB
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3n}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || { tail -20 gpurun_out/${P}_smoke.txt; exit 1; }
tail -1 gpurun_out/${P}_smoke.txt | cut -c1-120
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_exact.json 2> gpurun_out/${P}_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['ms_per_step'])"
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { grep -v amdgpu.ids gpurun_out/${P}_bench.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'])"
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera.json 2> gpurun_out/${P}_tera.err || { tail -20 gpurun_out/${P}_tera.err; exit 1; }
tail -1 gpurun_out/${P}_tera.json | cut -c1-300

# round 3 (late): TeraSort v4 with the radix window under the group's common
# key prefix (4 passes), refine v2 with 2-row Elkan steps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3m}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_terasort.py tests/test_kmeans_exact.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
timeout -k 10 240 python tools/kbench_exact.py > gpurun_out/${P}_kx.json 2> gpurun_out/${P}_kx.err || { tail -20 gpurun_out/${P}_kx.err; exit 1; }
tail -1 gpurun_out/${P}_kx.json | cut -c1-400
for B in 32 48; do
  timeout -k 10 300 env HBMR_TERA_SORT_BITS=$B python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera_b$B.json 2> gpurun_out/${P}_tera_b$B.err || { tail -20 gpurun_out/${P}_tera_b$B.err; exit 1; }
  echo "bits $B"; tail -1 gpurun_out/${P}_tera_b$B.json | cut -c1-330
done
timeout -k 10 300 python bench.py --exact --steps 10 --warmup 3 > gpurun_out/${P}_exact.json 2> gpurun_out/${P}_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_exact.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['ms_per_step'])"

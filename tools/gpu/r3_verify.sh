# round 3: verify the current tree on the GPU — the full GPU test suite, the
# default bench, the exact and file-backed variants, TeraSort v4 (opt-in), and
# the many-core rehearsal with the control-plane sampler at 8 ranks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3k}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/${P}_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${P}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || exit 1
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['phases_ms'])"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --exact > gpurun_out/${P}_bench_exact.json 2> gpurun_out/${P}_bench_exact.err || { tail -5 gpurun_out/${P}_bench_exact.err; exit 1; }
tail -1 gpurun_out/${P}_bench_exact.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('exact', d['dtype'], d['ms_per_step'], d['phases_ms'])"
timeout -k 10 300 python tools/write_kmeans_input.py --dir /tmp/km100m > gpurun_out/${P}_write_input.txt 2>&1 || { tail -5 gpurun_out/${P}_write_input.txt; exit 1; }
tail -1 gpurun_out/${P}_write_input.txt
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --input /tmp/km100m > gpurun_out/${P}_bench_file.json 2> gpurun_out/${P}_bench_file.err || { tail -5 gpurun_out/${P}_bench_file.err; exit 1; }
tail -1 gpurun_out/${P}_bench_file.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file', d['ms_per_step'], d['warmup_seconds'], d['phases_ms'])"
rm -rf /tmp/km100m
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera100_v3.json 2> gpurun_out/${P}_tera100_v3.err || { tail -5 gpurun_out/${P}_tera100_v3.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v3.json
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 -D hbmr.terasort.reduce.gid=true > gpurun_out/${P}_tera100_v4.json 2> gpurun_out/${P}_tera100_v4.err || { tail -5 gpurun_out/${P}_tera100_v4.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v4.json

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log | cut -c1-200 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1b.log 2>&1 && tail -1 gpurun_out/bench1b.log | cut -c1-200 && \
timeout -k 10 600 python -u tools/bench_file_load.py --points 100000000 --files 64 --maps 128 --load-threads 16 --out gpurun_out/file_load_100m.json > gpurun_out/file_load_100m.log 2>&1; rc=$?; tail -5 gpurun_out/file_load_100m.log | cut -c1-400; exit $rc

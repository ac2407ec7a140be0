set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
df -h /tmp | tail -1; free -g | head -2
HBMR_TRACE='gpurun_out/trace_bench_{rank}.jsonl' HBMR_WORKER_CLEAN_EXIT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_trace.log 2>&1; tail -1 gpurun_out/bench_trace.log | cut -c1-200
timeout -k 10 400 python -u tools/bench_file_load.py --points 20000000 --files 16 --maps 32 --load-threads 16 > gpurun_out/file_load_20m.log 2>&1; rc=$?; tail -4 gpurun_out/file_load_20m.log; exit $rc

# 1-GPU bench with control-plane tracing (rank process + worker) and a kernel trace of the worker
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HBMR_TRACE='gpurun_out/trace_bench_{rank}.jsonl' HBMR_WORKER_CLEAN_EXIT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_trace.log 2>&1 && tail -1 gpurun_out/bench_trace.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_worker -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_worker.log 2>&1 && tail -1 gpurun_out/prof_worker.log | cut -c1-300 && find gpurun_out/prof_worker -name '*.csv' | head

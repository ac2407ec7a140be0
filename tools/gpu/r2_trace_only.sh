# 1-GPU bench with control-plane tracing of the rank process and its GPU worker
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HBMR_TRACE='gpurun_out/trace_bench_{rank}.jsonl' HBMR_WORKER_CLEAN_EXIT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_trace.log 2>&1; tail -1 gpurun_out/bench_trace.log | cut -c1-300

set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log | cut -c1-200 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1b.log 2>&1 && tail -1 gpurun_out/bench1b.log | cut -c1-200 && \
HBMR_TRACE='gpurun_out/trace_bench_{rank}.jsonl' HBMR_WORKER_CLEAN_EXIT=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_trace.log 2>&1; tail -1 gpurun_out/bench_trace.log | cut -c1-200
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc

# GPU tests + 1-GPU bench (worker mode) + kernel-trace profile of the worker-mode bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -3 gpurun_out/pytest_gpu.log && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log | cut -c1-600 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_worker -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_worker.log 2>&1 && tail -1 gpurun_out/prof_worker.log | cut -c1-300

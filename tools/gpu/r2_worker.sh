# GPU tests + bench with per-rank GPU worker processes (default) + in-process + 2-rank shared device
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log | cut -c1-300 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --in-process > gpurun_out/bench1_inproc.log 2>&1 && tail -1 gpurun_out/bench1_inproc.log | cut -c1-300 && \
HBMR_SHARED_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench2_shared.log 2>&1 && tail -1 gpurun_out/bench2_shared.log | cut -c1-300

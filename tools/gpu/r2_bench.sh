# 1-GPU bench + 2-rank shared-device rehearsal (gloo) of the multi-process path
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && tail -1 gpurun_out/bench1.log | cut -c1-400 && \
HBMR_SHARED_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/bench2_shared.log 2>&1 && tail -1 gpurun_out/bench2_shared.log | cut -c1-600

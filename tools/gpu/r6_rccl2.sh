#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29711 tools/rccl_two_ranks_one_gpu.py > gpurun_out/r6_rccl2.txt 2>&1
echo "RCCL2_EXIT $?"
tail -20 gpurun_out/r6_rccl2.txt

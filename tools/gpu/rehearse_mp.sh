# multi-process rehearsal on a 1-GPU box: 2 ranks share GPU 0, gloo collectives
set -o pipefail
mkdir -p gpurun_out
HBMR_TRACE='gpurun_out/mp2_trace_r{rank}.json' HBMR_SHARED_DEVICE=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 ${BENCH_ARGS:-} > gpurun_out/rehearse_mp2.log 2>&1
echo EXIT $?
tail -2 gpurun_out/rehearse_mp2.log

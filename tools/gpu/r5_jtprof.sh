# JobTracker-process sampling profile + RPC method stats at N ranks (CPU rehearsal)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/jtprof
P=${P:-r5j}
n=${N:-8}
HBMR_SAMPLE_PROF=$PWD/gpurun_out/jtprof/${P} timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus $n --simulate-ms 0.26 --steps 40 --warmup 5 -D hbmr.jobtracker.process=true > gpurun_out/${P}_n${n}.json 2> gpurun_out/${P}_n${n}.err || { tail -5 gpurun_out/${P}_n${n}.err; exit 1; }
tail -c 400 gpurun_out/${P}_n${n}.json

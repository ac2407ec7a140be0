# cProfile of every thread of the JobTracker process in the 8-rank rehearsal (HBMR_CPROFILE)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=${P:-r5jc}
mkdir -p gpurun_out/$P
HBMR_CPROFILE=$PWD/gpurun_out/$P/p timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29557 bench.py --gpus 8 --simulate-ms 0.26 --steps 60 --warmup 5 -D hbmr.jobtracker.process=true > gpurun_out/$P/n8.json 2> gpurun_out/$P/n8.err || { tail -5 gpurun_out/$P/n8.err; exit 1; }
f=$(grep -l "jobtracker.py" gpurun_out/$P/p_*.txt | head -1)
echo "JT profile: $f"
cp ${f%.txt}.prof gpurun_out/$P/jt.prof
rm -f gpurun_out/$P/p_*

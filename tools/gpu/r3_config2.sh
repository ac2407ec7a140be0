# round 3: config 2 (Pipes GPU K-Means 1M x 128, k=64, 8 maps, one GPU slot)
# traced at 2 (default), 4 and 8 concurrent Pipes children per slot
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3c2}
for c in 2 4 8; do
  timeout -k 10 200 python tools/trace_config2.py --gpu -D hbmr.gpu.pipes.concurrency=$c > gpurun_out/${P}_c$c.txt 2>&1 || { tail -20 gpurun_out/${P}_c$c.txt; exit 1; }
  echo "concurrency $c"; grep "iteration" gpurun_out/${P}_c$c.txt
done

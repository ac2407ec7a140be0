# TeraSort: 100 GB in HBM, 100 GB with output committed to /dev/shm, and an
# out-of-core run (data 2.5x the HBM budget)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4t}
df -h /dev/shm /tmp | tail -2
free -g | head -2
timeout -k 10 400 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 2 --output /dev/shm/tera-out > gpurun_out/${P}_100g.json 2> gpurun_out/${P}_100g.err || { tail -20 gpurun_out/${P}_100g.err; rm -rf /dev/shm/tera-out; exit 1; }
rm -rf /dev/shm/tera-out
tail -1 gpurun_out/${P}_100g.json | cut -c1-700
timeout -k 10 300 python tools/bench_terasort.py --rows 200000000 --split-rows 10000000 --steps 2 -D hbmr.terasort.hbm.budget.gb=8 > gpurun_out/${P}_ooc.json 2> gpurun_out/${P}_ooc.err || { tail -20 gpurun_out/${P}_ooc.err; exit 1; }
tail -1 gpurun_out/${P}_ooc.json | cut -c1-700

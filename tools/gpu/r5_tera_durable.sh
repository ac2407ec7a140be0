# TeraSort with the output committed (fsync per part, TeraOutputFormat) to the box's
# disk-backed overlay root, sized to its free space; and the 100 GB in-HBM sort
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5td}
timeout -k 10 600 python3 tools/bench_terasort.py --rows 1000000000 --steps 3 > gpurun_out/${P}_100g.json 2> gpurun_out/${P}_100g.err || { tail -5 gpurun_out/${P}_100g.err; exit 1; }
tail -c 400 gpurun_out/${P}_100g.json; echo
D=$GRAFT_REPO_ROOT/tera-out-durable
FREE=$(python3 -c "import shutil;print(shutil.disk_usage('$GRAFT_REPO_ROOT').free)")
ROWS=$(python3 -c "print(min(1000000000, int($FREE/100/1.3)//10000000*10000000))")
echo "durable: $(stat -f -c %T $GRAFT_REPO_ROOT) free=$FREE rows=$ROWS"
timeout -k 10 900 python3 tools/bench_terasort.py --rows $ROWS --steps 1 --warmup 1 --output $D > gpurun_out/${P}_durable.json 2> gpurun_out/${P}_durable.err || { tail -5 gpurun_out/${P}_durable.err; rm -rf $D; exit 1; }
rm -rf $D
tail -c 700 gpurun_out/${P}_durable.json

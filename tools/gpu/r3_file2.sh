# round 3: TeraSort 100 GB v3 and v4 (packed-id reduce), then the file-backed
# K-Means bench at 20M points with thread stacks dumped every 25 s (the first
# attempt never finished its first iteration)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3o}
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera100_v3.json 2> gpurun_out/${P}_tera100_v3.err || { tail -5 gpurun_out/${P}_tera100_v3.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v3.json | cut -c1-300
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 -D hbmr.terasort.reduce.gid=true > gpurun_out/${P}_tera100_v4.json 2> gpurun_out/${P}_tera100_v4.err || { tail -5 gpurun_out/${P}_tera100_v4.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v4.json | cut -c1-300
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km20m --points 20000000 > gpurun_out/${P}_write20.txt 2>&1 || { tail -5 gpurun_out/${P}_write20.txt; exit 1; }
tail -1 gpurun_out/${P}_write20.txt
HBMR_STACKDUMP_S=25 timeout -k 10 110 python bench.py --steps 5 --warmup 2 --verbose --input /tmp/km20m --points 20000000 > gpurun_out/${P}_bench_file20.json 2> gpurun_out/${P}_bench_file20.err
rc=$?
grep "bench:" gpurun_out/${P}_bench_file20.err
echo "file20 rc=$rc"
[ $rc -eq 0 ] && tail -1 gpurun_out/${P}_bench_file20.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file20', d['ms_per_step'], d['warmup_seconds'], d['cpu_maps'], d['cost_model'])"
exit $rc

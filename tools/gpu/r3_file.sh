# round 3: exact-mode kernel timings, the file-backed K-Means bench (SequenceFile input -> HBM) at 20M then
# 100M points with warmup progress on stderr, then TeraSort 100 GB v3 and v4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3l}
timeout -k 10 150 python tools/kbench_exact.py > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { grep -v amdgpu.ids gpurun_out/${P}_kbench_exact.err | tail -20; exit 1; }
cat gpurun_out/${P}_kbench_exact.json
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km20m --points 20000000 > gpurun_out/${P}_write20.txt 2>&1 || { tail -5 gpurun_out/${P}_write20.txt; exit 1; }
tail -1 gpurun_out/${P}_write20.txt
timeout -k 10 170 python bench.py --steps 5 --warmup 2 --verbose --input /tmp/km20m --points 20000000 > gpurun_out/${P}_bench_file20.json 2> gpurun_out/${P}_bench_file20.err || { grep -v amdgpu.ids gpurun_out/${P}_bench_file20.err | tail -20; exit 1; }
grep "bench:" gpurun_out/${P}_bench_file20.err
tail -1 gpurun_out/${P}_bench_file20.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file20', d['ms_per_step'], d['warmup_seconds'], d['cpu_maps'], d['cost_model'])"
rm -rf /tmp/km20m
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera100_v3.json 2> gpurun_out/${P}_tera100_v3.err || { tail -5 gpurun_out/${P}_tera100_v3.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v3.json | cut -c1-400
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 -D hbmr.terasort.reduce.gid=true > gpurun_out/${P}_tera100_v4.json 2> gpurun_out/${P}_tera100_v4.err || { tail -5 gpurun_out/${P}_tera100_v4.err; exit 1; }
tail -1 gpurun_out/${P}_tera100_v4.json | cut -c1-400
timeout -k 10 120 python tools/write_kmeans_input.py --dir /tmp/km100m > gpurun_out/${P}_write100.txt 2>&1 || { tail -5 gpurun_out/${P}_write100.txt; exit 1; }
tail -1 gpurun_out/${P}_write100.txt
timeout -k 10 170 python bench.py --steps 5 --warmup 2 --verbose --input /tmp/km100m > gpurun_out/${P}_bench_file100.json 2> gpurun_out/${P}_bench_file100.err || { grep -v amdgpu.ids gpurun_out/${P}_bench_file100.err | tail -20; exit 1; }
grep "bench:" gpurun_out/${P}_bench_file100.err
tail -1 gpurun_out/${P}_bench_file100.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('file100', d['ms_per_step'], d['warmup_seconds'], d['cpu_maps'], d['cost_model'])"

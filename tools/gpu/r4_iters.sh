set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4it}
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_w -o run -- python3 bench.py > gpurun_out/${P}.log 2>&1 || { tail -20 gpurun_out/${P}.log; exit 1; }
grep '"metric"' gpurun_out/${P}.log | cut -c1-150
DB=$(ls -S $(find /tmp/${P}_w -name "*.db") | head -1)
python tools/iter_kernels.py $DB > gpurun_out/${P}_iters.txt 2>&1; cat gpurun_out/${P}_iters.txt
rm -rf /tmp/${P}_w
for i in 1 2; do
for v in 32 16; do
timeout -k 10 300 python bench.py -D hbmr.gpu.batch.target.unstaged=$v > gpurun_out/${P}_u${v}_$i.json 2> gpurun_out/${P}_u${v}_$i.err || { tail -20 gpurun_out/${P}_u${v}_$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_u${v}_$i.json').read().strip().splitlines()[-1]); print('unstaged=$v', d['ms_per_step'], d['release_to_finish_ms_per_job'][:3])"
done
done

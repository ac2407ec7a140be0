# round 3: 8-rank CPU rehearsal with rank-0 per-thread CPU and RPC counts
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3z}
HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= HBMR_SAMPLE_PROF_INTERVAL=1.0 HBMR_SAMPLE_PROF=gpurun_out/${P}_sp8 timeout -k 10 200 python bench.py --gpus 8 --simulate-ms 0.24 --steps 60 --warmup 3 > gpurun_out/${P}_n8.json 2> gpurun_out/${P}_n8.err || { tail -5 gpurun_out/${P}_n8.err; exit 1; }
tail -1 gpurun_out/${P}_n8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=8', d['ms_per_step'], d['rank0_cpu_ms_per_step'], d['phases_ms'])"
f=$(ls -S gpurun_out/${P}_sp8_* | head -1)
sed -n '/RPC server/,/inclusive/p' $f

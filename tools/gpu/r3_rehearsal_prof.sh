# round 3: the 8-rank CPU rehearsal with the control-plane stack sampler on
# every rank (HBMR_SAMPLE_PROF), reports under gpurun_out/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3k}
HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= HBMR_SAMPLE_PROF=gpurun_out/${P}_sp8 timeout -k 10 200 python bench.py --gpus 8 --simulate-ms 0.24 --steps 30 --warmup 3 > gpurun_out/${P}_sim8p.json 2> gpurun_out/${P}_sim8p.err || { tail -5 gpurun_out/${P}_sim8p.err; exit 1; }
tail -1 gpurun_out/${P}_sim8p.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=8', d['ms_per_step'], d['phases_ms'])"

# round 3: the control-plane changes (report RPC, lazy purges, targeted kicks)
# on the GPU: full GPU tests, the bench, then the 1/2/4/8-rank CPU rehearsal
# with rank-0 CPU per job
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3y}
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_gpu_tests.txt
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { grep -v amdgpu.ids gpurun_out/${P}_bench.err | tail -20; exit 1; }
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['rank0_cpu_ms_per_step'])"
echo "nproc $(nproc)"
for N in 1 2 4 8; do
  HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= timeout -k 10 200 python bench.py --gpus $N --simulate-ms 0.24 --steps 30 --warmup 3 > gpurun_out/${P}_n$N.json 2> gpurun_out/${P}_n$N.err || { echo "N=$N failed"; tail -5 gpurun_out/${P}_n$N.err; exit 1; }
  tail -1 gpurun_out/${P}_n$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N=$N', d['ms_per_step'], d['rank0_cpu_ms_per_step'], d['phases_ms'])"
done

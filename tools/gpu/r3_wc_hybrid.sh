# round 3: GPU WordCount over text files, cold + warm jobs, with 0 and 8 CPU
# map slots next to the GPU (hybrid scheduling): does the cost model give the
# CPU slots a share when the GPU tasks include loading their splits?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3wc}
for c in 0 8; do
  timeout -k 10 300 python tools/bench_configs.py wordcount-gpu --mb 2048 --files 32 --steps 2 --cpu-slots $c > gpurun_out/${P}_c$c.json 2> gpurun_out/${P}_c$c.err || { grep -v amdgpu.ids gpurun_out/${P}_c$c.err | tail -20; exit 1; }
  tail -1 gpurun_out/${P}_c$c.json | cut -c1-400
done

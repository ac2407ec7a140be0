set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_configs.py kmeans-pipes --points 1000000 --k 64 --files 8 --steps 6 > gpurun_out/config2.log 2>&1 && tail -1 gpurun_out/config2.log && \
timeout -k 10 300 python tools/trace_config2.py --gpu > gpurun_out/trace_config2.log 2>&1 && head -6 gpurun_out/trace_config2.log

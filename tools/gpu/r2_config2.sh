set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_pipes.py tests/test_pipes.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pipes.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pipes.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python tools/bench_configs.py kmeans-pipes --points 1000000 --k 64 --files 8 --steps 6 > gpurun_out/config2.log 2>&1 && tail -1 gpurun_out/config2.log && \
timeout -k 10 400 python tools/bench_configs.py kmeans-pipes --points 10000000 --k 64 --files 32 --steps 3 > gpurun_out/config2_10m.log 2>&1 && tail -1 gpurun_out/config2_10m.log

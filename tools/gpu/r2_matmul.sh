# config 4: matmul GPU tests, job bench with the hbmr GEMM and with hipBLASLt, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matmul.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_matmul.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_matmul.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_matmul.py --steps 10 > gpurun_out/matmul_hbmr.log 2>&1 && tail -1 gpurun_out/matmul_hbmr.log && \
timeout -k 10 300 python tools/bench_matmul.py --steps 10 --gemm hipblaslt > gpurun_out/matmul_hblt.log 2>&1 && tail -1 gpurun_out/matmul_hblt.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mm -o run -- python3 tools/bench_matmul.py --steps 5 > gpurun_out/prof_mm.log 2>&1 && tail -1 gpurun_out/prof_mm.log

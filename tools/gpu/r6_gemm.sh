set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_matmul.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] && timeout -k 10 300 python -u tools/bench_gemm_ab.py 8192 4096 > gpurun_out/gemm_ab.json 2> gpurun_out/gemm_ab.err; echo "ab rc=$?"; cat gpurun_out/gemm_ab.json

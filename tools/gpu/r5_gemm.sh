# GEMM variants A/B at 8192^3 vs hipBLASLt (tools/bench_gemm_ab.py), then the variant tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_matmul.py -m gpu -k "variants or layout" > gpurun_out/r5_gemm_tests.log 2>&1 || { tail -20 gpurun_out/r5_gemm_tests.log; exit 1; }
tail -2 gpurun_out/r5_gemm_tests.log
timeout -k 10 300 python3 tools/bench_gemm_ab.py > gpurun_out/r5_gemm_ab.json 2> gpurun_out/r5_gemm_ab.err || { tail -5 gpurun_out/r5_gemm_ab.err; exit 1; }
cat gpurun_out/r5_gemm_ab.json

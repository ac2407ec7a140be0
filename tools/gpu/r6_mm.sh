# config 4 (round 6 kernel): matmul job (65536x8192x8192 as 8 map tasks) with hipBLASLt vs the hand kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P=${P:-r6mm}
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_matmul.py -m gpu -k "job" > gpurun_out/${P}_tests.log 2>&1 || { tail -20 gpurun_out/${P}_tests.log; exit 1; }
tail -1 gpurun_out/${P}_tests.log
for g in hipblaslt hbmr; do
  timeout -k 10 300 python3 tools/bench_matmul.py --gemm $g > gpurun_out/${P}_$g.json 2> gpurun_out/${P}_$g.err || { tail -5 gpurun_out/${P}_$g.err; exit 1; }
  tail -c 500 gpurun_out/${P}_$g.json; echo
done

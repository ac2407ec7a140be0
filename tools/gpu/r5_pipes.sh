# Pipes K-Means: GPU tests (exact binary, shared child) + config 2 timing
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5p}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmeans_pipes.py -m gpu > gpurun_out/${P}_pipes_tests.log 2>&1 || { tail -40 gpurun_out/${P}_pipes_tests.log; exit 1; }
tail -3 gpurun_out/${P}_pipes_tests.log
timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 6 > gpurun_out/${P}_config2_exact.json 2> gpurun_out/${P}_config2_exact.err || { tail -20 gpurun_out/${P}_config2_exact.err; exit 1; }
cat gpurun_out/${P}_config2_exact.json
timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 6 --no-exact > gpurun_out/${P}_config2_bf16.json 2> gpurun_out/${P}_config2_bf16.err || { tail -20 gpurun_out/${P}_config2_bf16.err; exit 1; }
cat gpurun_out/${P}_config2_bf16.json

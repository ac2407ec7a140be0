# Pipes K-Means after the centroid-image buffer reuse: tests, config 2, trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5p2}
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kmeans_pipes.py -m gpu > gpurun_out/${P}_pipes_tests.log 2>&1 || { tail -40 gpurun_out/${P}_pipes_tests.log; exit 1; }
tail -3 gpurun_out/${P}_pipes_tests.log
timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 6 > gpurun_out/${P}_config2_exact.json 2> gpurun_out/${P}_config2_exact.err || { tail -20 gpurun_out/${P}_config2_exact.err; exit 1; }
cat gpurun_out/${P}_config2_exact.json
timeout -k 10 300 python3 -u tools/trace_config2.py --gpu > gpurun_out/${P}_trace.txt 2> gpurun_out/${P}_trace.err || { tail -20 gpurun_out/${P}_trace.err; exit 1; }
tail -40 gpurun_out/${P}_trace.txt

# Config 3 through the Pipes GPU binary: Pipes GPU tests, a traced k=1024
# iteration, then the 100M x 128 k=1024 comparison with the split job
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-c3}
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmeans_pipes.py -m gpu > gpurun_out/${P}_tests.log 2>&1 || { tail -30 gpurun_out/${P}_tests.log; exit 1; }
tail -1 gpurun_out/${P}_tests.log
timeout -k 10 300 python3 -u tools/trace_config2.py --gpu --k 1024 --files 16 > gpurun_out/${P}_trace.txt 2> gpurun_out/${P}_trace.err || { tail -20 gpurun_out/${P}_trace.err; exit 1; }
head -4 gpurun_out/${P}_trace.txt
timeout -k 10 ${C3T:-900} python3 -u tools/bench_config3_pipes.py --points ${C3N:-100000000} --files ${C3F:-128} --iters 4 --dir /tmp/c3data --out gpurun_out/${P}_result.json > gpurun_out/${P}_run.txt 2> gpurun_out/${P}_run.err || { tail -20 gpurun_out/${P}_run.err; tail -5 gpurun_out/${P}_run.txt; exit 1; }
tail -1 gpurun_out/${P}_run.txt

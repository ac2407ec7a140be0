# 2-rank shared-GPU device-collective test, bench x2, kernel-trace profile of the worker-mode bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_multirank.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_multirank.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1a.log 2>&1 && tail -1 gpurun_out/bench1a.log | cut -c1-300 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1b.log 2>&1 && tail -1 gpurun_out/bench1b.log | cut -c1-300 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_worker -o run -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof_worker.log 2>&1 && tail -1 gpurun_out/prof_worker.log | cut -c1-300 && ls -R gpurun_out/prof_worker | head -20

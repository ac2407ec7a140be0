set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_terasort.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_terasort.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_terasort.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python tools/bench_terasort.py --rows 100000000 --steps 3 > gpurun_out/terasort_10g.log 2>&1 && tail -1 gpurun_out/terasort_10g.log && \
timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g.log 2>&1 && tail -1 gpurun_out/terasort_100g.log

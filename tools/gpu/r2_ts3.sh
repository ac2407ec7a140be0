set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g.log 2>&1; rc=$?; tail -1 gpurun_out/terasort_100g.log | cut -c1-700; exit $rc

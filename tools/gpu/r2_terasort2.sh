set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_terasort.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_terasort.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_terasort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g.log 2>&1; rc=$?; tail -1 gpurun_out/terasort_100g.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 1 > gpurun_out/prof_ts.log 2>&1; tail -1 gpurun_out/prof_ts.log | cut -c1-300

# multi-record gather v2: GPU sort tests, then TeraSort 100 GB with v1 and v2 gathers
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_terasort.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_terasort_gather.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_terasort_gather.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g_g2.log 2>&1; rc=$?; tail -1 gpurun_out/terasort_100g_g2.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc
HBMR_GATHER_V1=1 timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g_g1.log 2>&1; rc=$?; tail -1 gpurun_out/terasort_100g_g1.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts4 -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 2 > gpurun_out/prof_ts4.log 2>&1; tail -1 gpurun_out/prof_ts4.log | cut -c1-300

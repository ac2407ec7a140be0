# TeraSort: 100 GB timing (v2 radix) and a kernel profile of a 20 GB sort
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_terasort.py --rows 1000000000 --steps 2 > gpurun_out/terasort_100g_v2.log 2>&1; rc=$?; tail -1 gpurun_out/terasort_100g_v2.log | cut -c1-700; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts3 -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 2 > gpurun_out/prof_ts3.log 2>&1; tail -1 gpurun_out/prof_ts3.log | cut -c1-300

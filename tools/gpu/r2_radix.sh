# radix sort v1 vs v2 kernels: correctness (10M) and speed (100M, 1000M), GPU tests of the sort
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/bench_radix.py --n 10000000 --reps 3 > gpurun_out/radix_v2_10m.log 2>&1; rc=$?; cat gpurun_out/radix_v2_10m.log | tail -3; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/bench_radix.py --n 10000000 --reps 3 --skew > gpurun_out/radix_v2_10m_skew.log 2>&1 && tail -1 gpurun_out/radix_v2_10m_skew.log && \
HBMR_RADIX_V1=1 timeout -k 10 120 python tools/bench_radix.py --n 100000000 --reps 3 --check 0 > gpurun_out/radix_v1_100m.log 2>&1 && tail -1 gpurun_out/radix_v1_100m.log && \
timeout -k 10 120 python tools/bench_radix.py --n 100000000 --reps 3 --check 0 > gpurun_out/radix_v2_100m.log 2>&1 && tail -1 gpurun_out/radix_v2_100m.log && \
timeout -k 10 300 python -u -m pytest tests/test_terasort.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_terasort_radix.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_terasort_radix.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_radix -o run -- python3 tools/bench_radix.py --n 100000000 --reps 2 --check 0 > gpurun_out/prof_radix.log 2>&1 && tail -1 gpurun_out/prof_radix.log

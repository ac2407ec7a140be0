# round 3: GPU tests of the delta combiner + pre-staging (stop at the first failure)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_kmeans_kernels.py tests/test_kmeans_job.py tests/test_gpu_worker.py > gpurun_out/r3c_tests.txt 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r3c_tests.txt | tail -8; tail -2 gpurun_out/r3c_tests.txt; exit $rc

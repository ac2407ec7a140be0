#!/bin/bash
# Round-6 GPU pass: the gpu test tier, then the default bench line.  A test
# failure (exit 1) still runs the bench; a time limit, abort or crash stops.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r6_gpu_tests.log 2>&1
rc=$?
echo "PYTEST_EXIT $rc"
tail -3 gpurun_out/r6_gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
rc2=$?
echo "BENCH_EXIT $rc2"
cat gpurun_out/r6_bench.json
exit $rc2

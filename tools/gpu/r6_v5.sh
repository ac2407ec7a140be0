#!/bin/bash
# v5 (barrier-free private-slot exact assign) vs v3: parity test + A/B timing
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_kmeans_exact.py -k "batch_labels_at_bench_shape" > gpurun_out/r6_v5_test.log 2>&1
rc=$?
echo "TEST_EXIT $rc"
tail -3 gpurun_out/r6_v5_test.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/kbench_v3.py --modes v3,v5,v3,v5,v2 --reps 9 > gpurun_out/r6_v5_ab.jsonl 2>&1
echo "AB_EXIT $?"
cat gpurun_out/r6_v5_ab.jsonl

#!/bin/bash
# barrier-free step-2 loop: exact-label tests, then A/B against the barrier path
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kmeans_exact.py -m gpu > gpurun_out/r6_q2_tests.log 2>&1
rc=$?
echo "TEST_EXIT $rc"; tail -2 gpurun_out/r6_q2_tests.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/r6_q2_ab.jsonl
for rep in 1 2 3; do
  for sync in 1 0; do
    HBMR_Q2_SYNC=$sync timeout -k 10 120 python3 -u tools/kbench_v3.py --modes v3 --reps 11 > gpurun_out/r6_q2.txt 2>&1 || { tail -5 gpurun_out/r6_q2.txt; exit 1; }
    python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r6_q2.txt') if l.startswith('{')][-1]
d['q2_sync']=$sync; print(json.dumps(d)); open('gpurun_out/r6_q2_ab.jsonl','a').write(json.dumps(d)+'\n')"
  done
done

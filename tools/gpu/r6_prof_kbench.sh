#!/bin/bash
# kernel durations of one exact batch (12.5M x 128, k=1024) on one stream
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_pk
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_pk -o kb -- python3 tools/kbench_v3.py --modes v3 --reps 9 > gpurun_out/r6_pk.txt 2> gpurun_out/r6_pk.err
rc=$?
echo "PROF_EXIT $rc"
cat gpurun_out/r6_pk.txt
find gpurun_out/r6_pk -name "*.csv" | head
exit $rc

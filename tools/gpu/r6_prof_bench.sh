#!/bin/bash
# kernel table of the bench line (rocprofv3 kernel trace + stats)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6_prof -o bench -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/r6_prof_bench.json 2> gpurun_out/r6_prof_bench.err
rc=$?
echo "PROF_EXIT $rc"
tail -1 gpurun_out/r6_prof_bench.json | cut -c1-300
find gpurun_out/r6_prof -name "*stats*" | head
exit $rc

#!/bin/bash
# Kernel table of TeraSort (20 GB, 2 timed sorts) under rocprofv3.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=${P:-r6tprof}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${P} -o run -- \
  python3 tools/bench_terasort.py --rows 200000000 --steps 2 > gpurun_out/${P}.json 2> gpurun_out/${P}.err
rc=$?
tail -1 gpurun_out/${P}.json
[ $rc -eq 0 ] || { tail -5 gpurun_out/${P}.err; exit $rc; }
echo "profile in gpurun_out/${P}"

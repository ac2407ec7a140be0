#!/bin/bash
# TeraSort after the packed-key onesweep reduce: GPU sort tests, then 100 GB in HBM.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
P=${P:-r6tera}
timeout -k 10 400 python -u -m pytest tests/test_terasort.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/${P}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${P}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u tools/bench_terasort.py --rows 1000000000 --steps 3 \
  > gpurun_out/${P}_100gb.json 2> gpurun_out/${P}_100gb.err
rc=$?
tail -2 gpurun_out/${P}_100gb.json
[ $rc -eq 0 ] || { tail -5 gpurun_out/${P}_100gb.err; exit $rc; }

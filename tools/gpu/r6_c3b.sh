#!/bin/bash
# Pipes GPU tests, then config 3 through the Pipes GPU binary
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kmeans_pipes.py -m gpu > gpurun_out/r6_c3b_tests.log 2>&1 || { tail -30 gpurun_out/r6_c3b_tests.log; exit 1; }
tail -1 gpurun_out/r6_c3b_tests.log
bash tools/gpu/r6_c3.sh

#!/bin/bash
# Config 3 through the Pipes GPU binary vs the split job (100M x 128, k=1024)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 ${C3T:-900} python3 -u tools/bench_config3_pipes.py --points ${C3N:-100000000} --files ${C3F:-128} --iters ${C3I:-5} --dir /tmp/c3data --out gpurun_out/r6_c3_result.json > gpurun_out/r6_c3_run.txt 2> gpurun_out/r6_c3_run.err || { tail -20 gpurun_out/r6_c3_run.err; tail -5 gpurun_out/r6_c3_run.txt; exit 1; }
tail -3 gpurun_out/r6_c3_run.txt
rm -rf /tmp/c3data

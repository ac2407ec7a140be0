#!/bin/bash
# traced config-2 iteration (Pipes K-Means 1M x 128, k=64, 8 GPU maps)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/trace_config2.py --gpu > gpurun_out/r6_c2_trace.txt 2> gpurun_out/r6_c2_trace.err || { tail -20 gpurun_out/r6_c2_trace.err; exit 1; }
head -3 gpurun_out/r6_c2_trace.txt; wc -l gpurun_out/r6_c2_trace.txt

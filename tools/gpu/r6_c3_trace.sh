#!/bin/bash
# traced Pipes K-Means iteration at k=1024 with 128 maps (host-side per-map cost)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/trace_config2.py --gpu --k 1024 --files 128 --points ${TP:-12800000} > gpurun_out/r6_c3_trace.txt 2> gpurun_out/r6_c3_trace.err || { tail -20 gpurun_out/r6_c3_trace.err; exit 1; }
grep -E "iteration|jt.assigned|reduce\.|tt.reduce|job_finished|centroids_read" gpurun_out/r6_c3_trace.txt | head -40

#!/bin/bash
# cProfile (thread CPU) of every thread of a Pipes K-Means run at k=1024, 128 maps
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
HBMR_CPROFILE=gpurun_out/r6_c3prof timeout -k 10 400 python3 -u tools/bench_configs.py kmeans-pipes --points 12800000 --files 128 --k 1024 --steps 10 > gpurun_out/r6_c3prof.json 2> gpurun_out/r6_c3prof.err || { tail -20 gpurun_out/r6_c3prof.err; exit 1; }
cut -c1-400 gpurun_out/r6_c3prof.json
ls gpurun_out/ | grep r6_c3prof

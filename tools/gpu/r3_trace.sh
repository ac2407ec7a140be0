# round 3: host trace + kernel trace of the in-process bench (pre-staged iterations)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
HBMR_TRACE=gpurun_out/r3e_trace.jsonl timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r3e_prof -o run -- python3 bench.py --in-process --steps 6 --warmup 3 > gpurun_out/r3e_prof.log 2>&1 && \
python tools/trace_merge.py $(find gpurun_out/r3e_prof -name "*.db" | head -1) gpurun_out/r3e_trace.jsonl --iters 2 > gpurun_out/r3e_merged.txt; tail -5 gpurun_out/r3e_merged.txt; wc -l gpurun_out/r3e_merged.txt

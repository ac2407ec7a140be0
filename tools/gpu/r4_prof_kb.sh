# kernel trace of the exact micro-bench (grouped top-3 + refine pieces)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4r}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 tools/kbench_exact.py --dtypes f16 --reps 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
grep mfma_dtype gpurun_out/${P}_prof.log | cut -c1-300

# q2 variant timing (diagnostic): 0 base, 1 no Q2 atomics, 2 fp32 math, 3 no row loads
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4j}
for v in 0 1 2 3; do
  HBMR_Q2_VARIANT=$v timeout -k 10 120 python tools/kbench_exact.py --dtypes f16 --reps 3 > gpurun_out/${P}_v$v.json 2> gpurun_out/${P}_v$v.err || { tail -20 gpurun_out/${P}_v$v.err; exit 1; }
  echo "v$v $(cut -c1-400 gpurun_out/${P}_v$v.json)"
done

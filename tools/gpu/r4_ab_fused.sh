# A/B on one box: step 1 fused into the top-3 epilogue vs a separate scan
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4ab}
for F in 1 0; do
  HBMR_EXACT_FUSED_Q1=$F timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kb_f$F.json 2> gpurun_out/${P}_kb_f$F.err || { tail -20 gpurun_out/${P}_kb_f$F.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${P}_kb_f$F.json').read().strip().splitlines()[-1]); print('kbench fused=$F', d['exact_batch_ms'], d['assign_top3_ms'])"
done
for R in 1 2 3; do for F in 1 0; do
  HBMR_EXACT_FUSED_Q1=$F timeout -k 10 300 python bench.py --steps 15 --warmup 3 > gpurun_out/${P}_b_f${F}_$R.json 2> gpurun_out/${P}_b_f${F}_$R.err || { tail -20 gpurun_out/${P}_b_f${F}_$R.err; exit 1; }
  tail -1 gpurun_out/${P}_b_f${F}_$R.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench fused=$F rep=$R', d['ms_per_step'], d['map_device_ms_per_job'])"
done; done

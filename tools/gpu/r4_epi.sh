# exact-mode assign epilogue A/B (top-2 per track vs running top-3) + PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4m}
timeout -k 10 200 python tools/kbench_exact.py --dtypes f16,bf16 --reps 3 > gpurun_out/${P}_trk.json 2> gpurun_out/${P}_trk.err || { tail -20 gpurun_out/${P}_trk.err; exit 1; }
cut -c1-260 gpurun_out/${P}_trk.json
HBMR_EXACT_EPI=top3 timeout -k 10 200 python tools/kbench_exact.py --dtypes f16,bf16 --reps 3 > gpurun_out/${P}_top3.json 2> gpurun_out/${P}_top3.err || { tail -20 gpurun_out/${P}_top3.err; exit 1; }
cut -c1-260 gpurun_out/${P}_top3.json
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/${P}_pmc -o run --output-format csv -- python3 tools/kbench_exact.py --dtypes f16 --reps 1 > gpurun_out/${P}_pmc.log 2>&1 || { tail -20 gpurun_out/${P}_pmc.log; exit 1; }
echo pmc-ok

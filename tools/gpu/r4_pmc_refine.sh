# PMC passes over the exact micro-bench (refine v3 q2 bottleneck hunt)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4h}
A="python3 tools/kbench_exact.py --dtypes f16 --reps 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d gpurun_out/${P}_pmc1 -o run --output-format csv -- $A > gpurun_out/${P}_pmc1.log 2>&1 || { tail -20 gpurun_out/${P}_pmc1.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR -d gpurun_out/${P}_pmc2 -o run --output-format csv -- $A > gpurun_out/${P}_pmc2.log 2>&1 || { tail -20 gpurun_out/${P}_pmc2.log; exit 1; }
ls -R gpurun_out/${P}_pmc1 | head

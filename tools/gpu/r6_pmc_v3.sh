#!/bin/bash
# PMC pass over the exact batch (v3 fused assign + refine q2/q3)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6_pmc
timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r6_pmc -o pmc -- python3 tools/kbench_v3.py --modes v3 --reps 3 > gpurun_out/r6_pmc.txt 2> gpurun_out/r6_pmc.err
rc=$?
echo "PMC_EXIT $rc"
cat gpurun_out/r6_pmc.txt
find gpurun_out/r6_pmc -name "*.csv" | head
exit $rc

# PMC passes over the v4 / v2 top-3 kernels (tools/kbench_v4.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc1 -o run -- python3 $R/tools/kbench_v4.py --arms v2,v4 --rounds 2 > $R/gpurun_out/v4pmc1.log 2>&1 || { tail -20 $R/gpurun_out/v4pmc1.log; exit 1; }
F=$(find /tmp/pmc1 -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_agg.py $F top3_v4 top3_grouped_v2 > $R/gpurun_out/v4pmc1.txt 2>&1; cat $R/gpurun_out/v4pmc1.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc2 -o run -- python3 $R/tools/kbench_v4.py --arms v2,v4 --rounds 2 > $R/gpurun_out/v4pmc2.log 2>&1 || { tail -20 $R/gpurun_out/v4pmc2.log; exit 1; }
F=$(find /tmp/pmc2 -name "*counter_collection.csv" | head -1)
python3 $R/tools/pmc_agg.py $F top3_v4 top3_grouped_v2 > $R/gpurun_out/v4pmc2.txt 2>&1; cat $R/gpurun_out/v4pmc2.txt

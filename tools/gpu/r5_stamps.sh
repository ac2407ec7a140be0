# per-phase cycles of the v3 fused exact assign (s_memtime stamps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5b}
timeout -k 10 300 python3 -u tools/kbench_v3.py --modes ${MODES:-v2,16} --stamps ${STAMPS:-48} > gpurun_out/${P}_stamps.log 2>&1; rc=$?; grep -E "mode|error|Error" gpurun_out/${P}_stamps.log; exit $rc

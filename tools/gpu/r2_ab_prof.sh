# kernel-level A/B: base worktree vs this tree (worker-mode bench under rocprofv3)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
(cd abtest/base && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../../gpurun_out/prof_base -o run -- python3 bench.py --in-process --steps 10 --warmup 3 > ../../gpurun_out/prof_base.log 2>&1) ; echo base rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o run -- python3 bench.py --in-process --steps 10 --warmup 3 > gpurun_out/prof_head.log 2>&1; echo head rc=$?
ls gpurun_out/prof_base gpurun_out/prof_head

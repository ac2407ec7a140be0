# end of session: every GPU test, smoke, default bench x2 and A/Bs, then the
# JobTracker-process sampler run
set -o pipefail
cd $GRAFT_REPO_ROOT
P=r4f bash tools/gpu/r4_final_a.sh || exit 1
bash tools/gpu/r4_jtprof.sh

# end-of-round validation, part B: TeraSort 100 GB with output, out-of-core,
# then the 1/2/4/8-rank CPU rehearsal on the box host
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4zb} bash tools/gpu/r4_tera.sh || exit 1
P=${P:-r4zb}r bash tools/gpu/r4_rehearse.sh

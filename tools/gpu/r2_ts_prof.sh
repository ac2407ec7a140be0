set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ts2 -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 1 > gpurun_out/prof_ts2.log 2>&1; tail -1 gpurun_out/prof_ts2.log | cut -c1-200

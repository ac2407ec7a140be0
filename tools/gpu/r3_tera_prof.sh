# round 3: kernel table of the 20 GB TeraSort with the packed-id reduce (v4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3x}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
tail -1 gpurun_out/${P}_prof.log | cut -c1-300
for db in $(find gpurun_out/${P}_prof -name "*.db"); do
  python tools/rocpd_summary.py $db --top 24 > gpurun_out/${P}_$(basename $db .db)_summary.md || true
done
ls gpurun_out/ | grep "${P}_.*summary" || true

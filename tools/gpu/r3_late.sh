# round 3 (late): config-2 Pipes concurrency sweep and the 100 GB TeraSort
# kernel table (csv stats: the rocpd db of a 1B-record run came back empty)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3l}
for c in 1 2 4 8; do
  timeout -k 10 200 python tools/trace_config2.py --gpu -D hbmr.gpu.pipes.concurrency=$c > gpurun_out/${P}_c2_c$c.txt 2>&1 || { tail -20 gpurun_out/${P}_c2_c$c.txt; exit 1; }
  echo "concurrency $c"; grep "iteration" gpurun_out/${P}_c2_c$c.txt
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${P}_tprof -o run -- python3 tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 2 > gpurun_out/${P}_tprof.log 2>&1 || { tail -20 gpurun_out/${P}_tprof.log; exit 1; }
grep '"metric"' gpurun_out/${P}_tprof.log | cut -c1-400
find gpurun_out/${P}_tprof -name "*kernel_stats.csv" | head -3
rm -f $(find gpurun_out/${P}_tprof -name "*kernel_trace.csv")

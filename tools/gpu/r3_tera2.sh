# round 3: TeraSort v4 with the 48-bit sort and the key-writing gather: GPU
# tests, 100 GB bench, 20 GB kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3t2}
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_terasort.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
timeout -k 10 300 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera100.json 2> gpurun_out/${P}_tera100.err || { tail -5 gpurun_out/${P}_tera100.err; exit 1; }
tail -1 gpurun_out/${P}_tera100.json | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 3 > gpurun_out/${P}_prof.log 2>&1 || { tail -20 gpurun_out/${P}_prof.log; exit 1; }
for db in $(find gpurun_out/${P}_prof -name "*.db"); do
  python tools/rocpd_summary.py $db --top 16 > gpurun_out/${P}_kernels.md || true
done
head -14 gpurun_out/${P}_kernels.md

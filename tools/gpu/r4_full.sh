# full GPU test suite, smoke, default bench (exact), fast-mode bench, then TeraSort runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4q}
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || { tail -20 gpurun_out/${P}_smoke.txt; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
tail -1 gpurun_out/${P}_bench.json | cut -c1-400
timeout -k 10 300 python bench.py --no-exact --steps 20 --warmup 3 > gpurun_out/${P}_bench_fast.json 2> gpurun_out/${P}_bench_fast.err || { tail -20 gpurun_out/${P}_bench_fast.err; exit 1; }
tail -1 gpurun_out/${P}_bench_fast.json | cut -c1-400
P=${P}t bash tools/gpu/r4_tera.sh

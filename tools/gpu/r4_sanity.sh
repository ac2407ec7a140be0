set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/r4san_tests.txt 2>&1 || { tail -30 gpurun_out/r4san_tests.txt; exit 1; }
tail -1 gpurun_out/r4san_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4san_smoke.txt 2>&1 || { tail -20 gpurun_out/r4san_smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py > gpurun_out/r4san_bench.json 2> gpurun_out/r4san_bench.err || { tail -20 gpurun_out/r4san_bench.err; exit 1; }
tail -1 gpurun_out/r4san_bench.json | cut -c1-250

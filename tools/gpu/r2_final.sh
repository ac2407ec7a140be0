# round-2 closing validation: full GPU suite, smoke, bench x2 (+ exact mode), kernel stats profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu_final.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --verbose > gpurun_out/bench_final_a.log 2> gpurun_out/bench_final_a.err && tail -1 gpurun_out/bench_final_a.log | cut -c1-400 && \
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_final_b.log 2>&1 && tail -1 gpurun_out/bench_final_b.log | cut -c1-400 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 10 --warmup 3 --in-process > gpurun_out/prof_final.log 2>&1 && tail -1 gpurun_out/prof_final.log | cut -c1-300

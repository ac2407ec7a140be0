# round 3: delta-combiner numerics + bench A/B (delta vs sorted) + in-process kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_kmeans_kernels.py tests/test_kmeans_job.py > gpurun_out/r3a_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r3a_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 10 --warmup 2 > gpurun_out/r3a_bench_delta.json 2> gpurun_out/r3a_bench_delta.err && tail -1 gpurun_out/r3a_bench_delta.json | cut -c1-300 && \
timeout -k 10 240 python bench.py --steps 10 --warmup 2 -D hbmr.kmeans.combiner=sorted > gpurun_out/r3a_bench_sorted.json 2> gpurun_out/r3a_bench_sorted.err && tail -1 gpurun_out/r3a_bench_sorted.json | cut -c1-300 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a_prof -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/r3a_prof.log 2>&1 && \
python tools/rocpd_summary.py $(find gpurun_out/r3a_prof -name "*.db" | head -1) --iterations --top 14 > gpurun_out/r3a_prof_summary.md && cat gpurun_out/r3a_prof_summary.md | tail -16

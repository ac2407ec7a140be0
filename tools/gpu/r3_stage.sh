# round 3: delta combiner + pre-staged iterations: GPU tests, bench A/B, in-process kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_kmeans_kernels.py tests/test_kmeans_job.py tests/test_gpu_worker.py > gpurun_out/r3b_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r3b_tests.txt; [ $rc -eq 0 ] || exit $rc
b() { timeout -k 10 240 python bench.py --steps 10 --warmup 2 "$@" 2> gpurun_out/r3b_$N.err > gpurun_out/r3b_$N.json && tail -1 gpurun_out/r3b_$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$N', d['ms_per_step'], d['phases_ms'])"; }
N=default b && N=sorted b -D hbmr.kmeans.combiner=sorted && N=noprestage b --no-prestage && N=r2like b --no-prestage --prefetch 1 -D hbmr.kmeans.combiner=sorted && N=default2 b && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3b_prof -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/r3b_prof.log 2>&1 && \
python tools/rocpd_summary.py $(find gpurun_out/r3b_prof -name "*.db" | head -1) --iterations --top 16 > gpurun_out/r3b_prof_summary.md && tail -14 gpurun_out/r3b_prof_summary.md

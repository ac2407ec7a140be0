# round 3: batch-size A/B of the pre-staged delta bench + GPU tests + host/kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3f}
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_kmeans_kernels.py tests/test_gpu_worker.py > gpurun_out/${P}_tests.txt 2>&1; rc=$?
tail -2 gpurun_out/${P}_tests.txt; [ $rc -eq 0 ] || exit $rc
b() { timeout -k 10 240 python bench.py --steps 10 --warmup 2 "$@" 2> gpurun_out/${P}_$N.err > gpurun_out/${P}_$N.json && tail -1 gpurun_out/${P}_$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$N', d['ms_per_step'], d['phases_ms'])"; }
N=t16 b && N=t64 b -D hbmr.gpu.batch.target=64 && N=t8 b -D hbmr.gpu.batch.target=8 && N=t16b b && N=inproc b --in-process && \
HBMR_TRACE=gpurun_out/${P}_trace.jsonl timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${P}_prof -o run -- python3 bench.py --in-process --steps 6 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 && \
python tools/trace_merge.py $(find gpurun_out/${P}_prof -name "*.db" | head -1) gpurun_out/${P}_trace.jsonl --iters 2 > gpurun_out/${P}_merged.txt; \
python tools/rocpd_summary.py $(find gpurun_out/${P}_prof -name "*.db" | head -1) --iterations --top 14 > gpurun_out/${P}_prof_summary.md; tail -8 gpurun_out/${P}_prof_summary.md

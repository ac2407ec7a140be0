# round 3 (part B): TeraSort v3 (20 GB rocprof, 100 GB, output-committed), config-2 Pipes
# trace, GEMM v2 A/B, 2-rank shared-device bench, many-core CPU rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3i}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_tera20 -o run -- python3 tools/bench_terasort.py --rows 200000000 --steps 2 > gpurun_out/${P}_tera20.json 2> gpurun_out/${P}_tera20.err || { tail -5 gpurun_out/${P}_tera20.err; exit 1; }
tail -1 gpurun_out/${P}_tera20.json
timeout -k 10 400 python tools/bench_terasort.py --rows 1000000000 --split-rows 10000000 --steps 3 > gpurun_out/${P}_tera100.json 2> gpurun_out/${P}_tera100.err || { tail -5 gpurun_out/${P}_tera100.err; exit 1; }
tail -1 gpurun_out/${P}_tera100.json
timeout -k 10 300 python tools/bench_terasort.py --rows 100000000 --split-rows 10000000 --steps 2 --output /tmp/tera-out > gpurun_out/${P}_tera10_out.json 2> gpurun_out/${P}_tera10_out.err || { tail -5 gpurun_out/${P}_tera10_out.err; exit 1; }
tail -1 gpurun_out/${P}_tera10_out.json
rm -rf /tmp/tera-out
timeout -k 10 200 python tools/trace_config2.py --gpu > gpurun_out/${P}_config2_trace.txt 2>&1 || { tail -5 gpurun_out/${P}_config2_trace.txt; exit 1; }
grep -E "iteration" gpurun_out/${P}_config2_trace.txt
HBMR_GEMM=2 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_matmul.py > gpurun_out/${P}_gemm2_tests.txt 2>&1 && tail -1 gpurun_out/${P}_gemm2_tests.txt && \
timeout -k 10 200 python tools/bench_matmul.py > gpurun_out/${P}_matmul_v1.json 2>&1 && tail -2 gpurun_out/${P}_matmul_v1.json && \
HBMR_GEMM=2 timeout -k 10 200 python tools/bench_matmul.py > gpurun_out/${P}_matmul_v2.json 2>&1 && tail -2 gpurun_out/${P}_matmul_v2.json || exit 1
HBMR_SHARED_DEVICE=0 timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/${P}_bench_2rank_shared.json 2> gpurun_out/${P}_bench_2rank_shared.err || { tail -5 gpurun_out/${P}_bench_2rank_shared.err; exit 1; }
tail -1 gpurun_out/${P}_bench_2rank_shared.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('2rank-shared', d['ms_per_step'], d['phases_ms'])"
P=${P}_sim bash tools/gpu/r3_rehearsal.sh

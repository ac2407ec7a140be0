set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_hybrid.json 2> gpurun_out/bench_hybrid.err && \
timeout -k 10 400 python -u bench.py --policy stock --steps 2 --warmup 1 > gpurun_out/policy_stock.json 2> gpurun_out/policy_stock.err && \
timeout -k 10 300 python -u tools/bench_configs.py wordcount --mb 32 --steps 2 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo EXIT $?
cat gpurun_out/bench_hybrid.json gpurun_out/policy_stock.json gpurun_out/cfg1.json; tail -2 gpurun_out/pytest_gpu.log

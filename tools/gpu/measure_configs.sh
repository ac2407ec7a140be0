# BASELINE configs 1/2, MRBench, and the paper's policy ratio (stock/optional vs hybrid)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_configs.py kmeans-pipes --points 1000000 --k 64 --dims 128 --files 8 --steps 3 > gpurun_out/cfg2.json 2> gpurun_out/cfg2.err && \
timeout -k 10 200 python -u tools/bench_configs.py mrbench --jobs 20 > gpurun_out/mrbench.json 2> gpurun_out/mrbench.err && \
timeout -k 10 300 python -u bench.py --policy stock --steps 2 --warmup 1 > gpurun_out/policy_stock.json 2> gpurun_out/policy_stock.err && \
timeout -k 10 300 python -u bench.py --policy optional --steps 5 --warmup 2 > gpurun_out/policy_optional.json 2> gpurun_out/policy_optional.err && \
timeout -k 10 300 python -u tools/bench_configs.py wordcount --mb 32 --steps 2 > gpurun_out/cfg1.json 2> gpurun_out/cfg1.err
echo EXIT $?
cat gpurun_out/cfg2.json gpurun_out/mrbench.json gpurun_out/policy_stock.json gpurun_out/policy_optional.json gpurun_out/cfg1.json

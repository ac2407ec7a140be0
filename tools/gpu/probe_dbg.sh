set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-slots 0 > gpurun_out/bench_nocpu.json 2> gpurun_out/bench_nocpu.err && \
HBMR_TRACE=gpurun_out/probe_trace.json timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err
echo EXIT $?
cat gpurun_out/bench_nocpu.json gpurun_out/bench_trace.json

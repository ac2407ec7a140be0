set -o pipefail
mkdir -p gpurun_out
echo "nproc $(nproc) affinity $(python -c 'import os;print(len(os.sched_getaffinity(0)))') quota $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_hybrid.json 2> gpurun_out/bench_hybrid.err && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 > gpurun_out/bench_hybrid2.json 2> gpurun_out/bench_hybrid2.err
echo EXIT $?
cat gpurun_out/bench_hybrid.json gpurun_out/bench_hybrid2.json

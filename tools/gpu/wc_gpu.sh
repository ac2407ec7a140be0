set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wordcount_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_wc.log 2>&1 && \
timeout -k 10 400 python -u tools/bench_configs.py wordcount-gpu --mb 2048 --files 16 --steps 3 > gpurun_out/wc_gpu.json 2> gpurun_out/wc_gpu.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wc -o wc -- python3 tools/bench_configs.py wordcount-gpu --mb 1024 --files 16 --steps 2 > gpurun_out/wc_prof.log 2>&1
echo EXIT $?
tail -12 gpurun_out/pytest_wc.log; cat gpurun_out/wc_gpu.json

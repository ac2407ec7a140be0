# Config 2 (Pipes) + GPU test suite + 1-GPU headline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5f}
timeout -k 10 300 python3 -u tools/bench_configs.py kmeans-pipes --steps 25 > gpurun_out/${P}_config2.json 2> gpurun_out/${P}_config2.err || { tail -20 gpurun_out/${P}_config2.err; exit 1; }
python3 -c "import json,statistics as s;d=json.load(open('gpurun_out/${P}_config2.json'));t=d['pipes_iteration_s'][3:];print('config2 median_ms', round(1e3*s.median(t),2), 'min_ms', round(1e3*min(t),2))"
timeout -k 10 300 python3 -u tools/trace_config2.py --gpu > gpurun_out/${P}_trace.txt 2> gpurun_out/${P}_trace.err || { tail -20 gpurun_out/${P}_trace.err; exit 1; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${P}_pytest.log 2>&1 || { tail -40 gpurun_out/${P}_pytest.log; exit 1; }
tail -3 gpurun_out/${P}_pytest.log
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || { tail -20 gpurun_out/${P}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${P}_bench.json'));print({k:d[k] for k in ('ms_per_step','value','dtype','map_device_ms_per_job','rank0_cpu_ms_per_step')})"

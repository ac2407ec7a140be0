set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4q}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kmeans_exact.py tests/test_kmeans_kernels.py > gpurun_out/${P}_tests.txt 2>&1 || { tail -30 gpurun_out/${P}_tests.txt; exit 1; }
tail -1 gpurun_out/${P}_tests.txt
timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench.json 2> gpurun_out/${P}_kbench.err || { tail -20 gpurun_out/${P}_kbench.err; exit 1; }
cut -c1-700 gpurun_out/${P}_kbench.json
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/${P}_bench$i.json 2> gpurun_out/${P}_bench$i.err || { tail -20 gpurun_out/${P}_bench$i.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/${P}_bench$i.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['release_to_finish_ms_per_job'], d.get('final_shift'))"
done

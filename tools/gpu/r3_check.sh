# round 3: full GPU test suite + default bench + many-core CPU rehearsal (1/2/4/8 ranks)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3h}
timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests \
  > gpurun_out/${P}_gpu_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/${P}_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --steps 20 --warmup 3 > gpurun_out/${P}_bench.json 2> gpurun_out/${P}_bench.err || exit 1
tail -1 gpurun_out/${P}_bench.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['ms_per_step'], d['phases_ms'])"
P=${P}_sim bash tools/gpu/r3_rehearsal.sh

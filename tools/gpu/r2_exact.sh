# exact K-Means mode: kernels tests, full GPU suite, fidelity profile on 10M points
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_exact.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pytest_exact.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_exact.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/kmeans_fidelity.py --points 10000000 --iters 3 --out gpurun_out/kmeans_fidelity.json > gpurun_out/fidelity.log 2>&1; rc=$?; tail -5 gpurun_out/fidelity.log | cut -c1-600; exit $rc

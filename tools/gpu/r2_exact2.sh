set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/kmeans_fidelity.py --points 10000000 --iters 3 --out gpurun_out/kmeans_fidelity.json > gpurun_out/fidelity.log 2>&1; rc=$?; tail -5 gpurun_out/fidelity.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_kmeans_exact.py::test_exact_mode_job_matches_fp64_lloyd > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc

set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kmeans_v4.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_v4.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -15 gpurun_out/pytest_v4.log
if [ $rc -eq 0 ]; then
  timeout -k 10 400 python -u tools/kbench_v4.py --rounds 7 > gpurun_out/kbench_v4.json 2> gpurun_out/kbench_v4.err
  echo "kbench rc=$?"
  cat gpurun_out/kbench_v4.json; tail -5 gpurun_out/kbench_v4.err
fi

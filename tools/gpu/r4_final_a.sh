# end-of-round validation, part A: every GPU test, smoke, the default bench
# (x2) and its A/Bs (one slot, no taper, step 1 unfused), exact kernel bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4z}
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/${P}_tests.txt 2>&1 || { tail -40 gpurun_out/${P}_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/${P}_tests.txt | tail -2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${P}_smoke.txt 2>&1 || { tail -20 gpurun_out/${P}_smoke.txt; exit 1; }
echo smoke ok
timeout -k 10 300 python tools/kbench_exact.py --dtypes f16 > gpurun_out/${P}_kbench_exact.json 2> gpurun_out/${P}_kbench_exact.err || { tail -20 gpurun_out/${P}_kbench_exact.err; exit 1; }
cut -c1-600 gpurun_out/${P}_kbench_exact.json
for V in default default2 oneslot notaper unfused; do
  case $V in
    default|default2) ARGS="" ; ENVV="" ;;
    oneslot) ARGS="--gpu-slots 1" ; ENVV="" ;;
    notaper) ARGS="-D hbmr.gpu.batch.taper=false" ; ENVV="" ;;
    unfused) ARGS="" ; ENVV="HBMR_EXACT_FUSED_Q1=0" ;;
  esac
  env $ENVV timeout -k 10 300 python bench.py --steps 10 --warmup 3 $ARGS > gpurun_out/${P}_bench_$V.json 2> gpurun_out/${P}_bench_$V.err || { tail -20 gpurun_out/${P}_bench_$V.err; exit 1; }
  tail -1 gpurun_out/${P}_bench_$V.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', d['ms_per_step'], d['phases_ms'], d['map_device_ms_per_job'])"
done

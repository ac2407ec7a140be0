# exact default bench: GPU slots / batch size sweep on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4sw}
for V in base s3 t8 t32 base2 s3b t8b t32b; do
  case $V in
    base|base2) ARGS="" ;;
    s3|s3b) ARGS="--gpu-slots 3" ;;
    t8|t8b) ARGS="-D hbmr.gpu.batch.target=8" ;;
    t32|t32b) ARGS="-D hbmr.gpu.batch.target=32" ;;
  esac
  timeout -k 10 300 python bench.py --steps 15 --warmup 3 $ARGS > gpurun_out/${P}_$V.json 2> gpurun_out/${P}_$V.err || { tail -20 gpurun_out/${P}_$V.err; exit 1; }
  tail -1 gpurun_out/${P}_$V.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', d['ms_per_step'], d['map_device_ms_per_job'])"
done

# 8-rank CPU rehearsal with the JobTracker process sampled (stack sampler)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/jts
HIP_VISIBLE_DEVICES= CUDA_VISIBLE_DEVICES= HBMR_SAMPLE_PROF=/tmp/jts/s HBMR_SAMPLE_PROF_INTERVAL=0.001 timeout -k 10 200 python bench.py --gpus 8 --simulate-ms 0.24 --steps 40 --warmup 3 -D hbmr.jobtracker.process=true > gpurun_out/r4jtp.json 2> gpurun_out/r4jtp.err || { tail -5 gpurun_out/r4jtp.err; exit 1; }
tail -1 gpurun_out/r4jtp.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['rank0_cpu_ms_per_step'], d.get('jobtracker_cpu_ms_per_step'))"
for f in /tmp/jts/s_*.txt; do if grep -q "jtprocess" $f; then cp $f gpurun_out/r4jtp_jt.txt; fi; done
ls /tmp/jts | head -3
head -60 gpurun_out/r4jtp_jt.txt

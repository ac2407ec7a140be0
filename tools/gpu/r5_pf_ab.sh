# prefetch (iteration jobs ahead) 2 vs 3: 8-rank rehearsal interleaved, then the 1-GPU bench with 3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r5pf}
: > gpurun_out/${P}.jsonl
for rep in 1 2 3; do
  for pf in 2 3; do
    timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29600 + rep * 10 + pf)) bench.py --gpus 8 --simulate-ms 0.26 --steps 40 --warmup 5 --prefetch $pf -D hbmr.jobtracker.process=true > gpurun_out/${P}_${pf}_${rep}.json 2> gpurun_out/${P}_${pf}_${rep}.err || { tail -5 gpurun_out/${P}_${pf}_${rep}.err; exit 1; }
    python3 -c "
import json
d=json.loads(open('gpurun_out/${P}_${pf}_${rep}.json').read().strip().splitlines()[-1])
r={'prefetch':$pf,'rep':$rep,'ms_per_step':d['ms_per_step'],'jt_cpu':d['jobtracker_cpu_ms_per_step'],'max_job_ms':max(d['release_to_finish_ms_per_job'])}
print(json.dumps(r)); open('gpurun_out/${P}.jsonl','a').write(json.dumps(r)+'\n')"
  done
done
for pf in 2 3; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --prefetch $pf > gpurun_out/${P}_gpu_${pf}.json 2> gpurun_out/${P}_gpu_${pf}.err || { tail -5 gpurun_out/${P}_gpu_${pf}.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${P}_gpu_${pf}.json').read().strip().splitlines()[-1]);print('gpu prefetch $pf', d['ms_per_step'], d['cost_model'])"
done

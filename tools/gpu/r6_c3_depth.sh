#!/bin/bash
# config 3 through Pipes: mux FIFO depth 8 (default) vs 32 vs 128 (split job skipped)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r6_c3_depth.jsonl

for d in 8 32 8 32; do
  timeout -k 10 300 python3 -u tools/bench_config3_pipes.py --iters 4 --skip-split-job --dir /tmp/c3data --out gpurun_out/r6_c3d.json -D hbmr.pipes.gpu.queue.depth=$d > gpurun_out/r6_c3d.txt 2> gpurun_out/r6_c3d.err || { tail -20 gpurun_out/r6_c3d.err; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/r6_c3d.json'))
r={'depth':$d,'pipes_iteration_ms':d['pipes_iteration_ms']}
print(json.dumps(r)); open('gpurun_out/r6_c3_depth.jsonl','a').write(json.dumps(r)+'\n')"
done
rm -rf /tmp/c3data

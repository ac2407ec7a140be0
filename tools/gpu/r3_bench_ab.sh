# round 3: bench A/B (delta/sorted combiner, pre-staged or not) + in-process kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r3d}
b() { timeout -k 10 240 python bench.py --steps 10 --warmup 2 "$@" 2> gpurun_out/${P}_$N.err > gpurun_out/${P}_$N.json && tail -1 gpurun_out/${P}_$N.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$N', d['ms_per_step'], d['phases_ms'])"; }
N=default b && N=sorted b -D hbmr.kmeans.combiner=sorted && N=noprestage b --no-prestage && N=r2like b --no-prestage --prefetch 1 -D hbmr.kmeans.combiner=sorted && N=default2 b && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${P}_prof -o run -- python3 bench.py --in-process --steps 8 --warmup 3 > gpurun_out/${P}_prof.log 2>&1 && \
python tools/rocpd_summary.py $(find gpurun_out/${P}_prof -name "*.db" | head -1) --iterations --top 16 > gpurun_out/${P}_prof_summary.md && tail -14 gpurun_out/${P}_prof_summary.md

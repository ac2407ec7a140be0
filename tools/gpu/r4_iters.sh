set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
P=${P:-r4it}
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${P}_w -o run -- python3 bench.py > gpurun_out/${P}.log 2>&1 || { tail -20 gpurun_out/${P}.log; exit 1; }
grep '"metric"' gpurun_out/${P}.log | cut -c1-150
DB=$(ls -S $(find /tmp/${P}_w -name "*.db") | head -1)
python tools/iter_kernels.py $DB > gpurun_out/${P}_iters.txt 2>&1; cat gpurun_out/${P}_iters.txt
rm -rf /tmp/${P}_w

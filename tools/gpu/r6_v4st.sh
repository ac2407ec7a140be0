set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/kbench_v4.py --arms v2,v4 --rounds 5 --stamps > gpurun_out/kbench_v4st.json 2> gpurun_out/kbench_v4st.err
echo "rc=$?"; cat gpurun_out/kbench_v4st.json; tail -3 gpurun_out/kbench_v4st.err

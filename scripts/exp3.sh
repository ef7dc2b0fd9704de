set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KB_ONLY=gcn16 KB_TRACE=1
timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb3_nat.json 2> gpurun_out/kb3_nat.err && \
KB_MORTON=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb3_morton.json 2> gpurun_out/kb3_morton.err
rc=$?
cat gpurun_out/kb3_*.json
exit $rc

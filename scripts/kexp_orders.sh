set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KB_ONLY=gcn16_full,gcn16_no_produce,gcn16_no_ext KB_TRACE=1 KB_CHECK=1
timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb11_nat.json 2> gpurun_out/kb11.err && \
KB_MORTON=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb11_mor.json 2>> gpurun_out/kb11.err && \
KB_BLOCK=4 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb11_b4.json 2>> gpurun_out/kb11.err
rc=$?; cat gpurun_out/kb11_*.json; exit $rc

set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python scripts/check_f16x3.py > gpurun_out/check.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/check.log | tail -4; if [ $rc -ne 0 ]; then exit $rc; fi
export KB_ONLY=gcn16,gcn_full KB_TRACE=1 KB_CHECK=1
timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb6_nat.json 2> gpurun_out/kb6_nat.err && \
KB_MORTON=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb6_morton.json 2> gpurun_out/kb6_morton.err
rc=$?
cat gpurun_out/kb6_*.json
exit $rc

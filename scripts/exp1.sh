set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export KB_ONLY=gcn_full,gcn_no_mfma,gcn_no_gather,linear_rows,linear_no_load,copy,diag_csr_gather,diag_copy
timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb_nat.json 2> gpurun_out/kb_nat.err && \
KB_MORTON=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb_morton.json 2> gpurun_out/kb_morton.err && \
KB_SHUFFLE=0 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb_shuf.json 2> gpurun_out/kb_shuf.err
rc=$?
cat gpurun_out/kb_*.json
exit $rc

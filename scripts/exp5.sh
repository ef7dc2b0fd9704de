set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
KB_ONLY=gcn16_full KB_CHECK=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb5_nat.json 2>gpurun_out/kb5.err && \
KB_ONLY=gcn16_full KB_CHECK=1 KB_MORTON=1 timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb5_mor.json 2>>gpurun_out/kb5.err
rc=$?; cat gpurun_out/kb5_*.json; if [ $rc -ne 0 ]; then tail gpurun_out/kb5.err; exit $rc; fi
export KB_ONLY=gcn16_full
bash scripts/pmc_cmd.sh gpurun_out/pmc16_nat scripts/kbench.py && PMC_SET=mem bash scripts/pmc_cmd.sh gpurun_out/pmc16_nat_mem scripts/kbench.py && \
python scripts/pmc_report.py gpurun_out/pmc16_nat && python scripts/pmc_report.py gpurun_out/pmc16_nat_mem

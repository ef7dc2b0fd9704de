set -u
mkdir -p gpurun_out/pmc9
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
KB_ONLY=gcn16_full,gcn16_plain,gcn16_no_produce timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb9_nat.json 2> gpurun_out/kb9.err && \
KB_MORTON=1 KB_ONLY=gcn16_full,gcn16_plain,gcn16_no_produce timeout -k 10 240 python scripts/kbench.py > gpurun_out/kb9_mor.json 2>> gpurun_out/kb9.err
rc=$?; cat gpurun_out/kb9_*.json; if [ $rc -ne 0 ]; then exit $rc; fi
for c in gcn16_no_produce_plain gcn16_no_produce; do
  for grp in "WRITE_SIZE" "FETCH_SIZE"; do
    KB_ONLY=$c timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc9/${c}_$grp -o run --output-format csv -- python scripts/kbench.py > gpurun_out/pmc9/${c}_$grp.log 2>&1 || exit 1
  done
done
python scripts/pmc_report.py "gpurun_out/pmc9/*" 2>&1 | grep -A3 gcn_f16x3

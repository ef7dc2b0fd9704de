#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only, no tracing
# domains) over an arbitrary python command:
#   scripts/pmc_cmd.sh <outdir> <python args...>
# Groups: MFMA busy + clocks, wave wait/issue breakdown, LDS, instruction mix.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
out=$1; shift
mkdir -p "$out"
i=0
if [ "${PMC_SET:-sq}" = mem ]; then
  PGROUPS=("TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
          "TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
          "TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_avr TCC_REQ_sum"
          "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
          "TA_BUSY_avr TA_TOTAL_WAVEFRONTS_sum" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum")
else
  PGROUPS=("SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAVES"
          "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
          "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS"
          "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA SQ_INSTS_VALU")
fi
for grp in "${PGROUPS[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$out/p$i" -o run --output-format csv \
      -- python "$@" > "$out/p$i.log" 2>&1
  rc=$?; echo "pmc pass $i ($grp) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/p$i.log"; exit $rc; fi
done

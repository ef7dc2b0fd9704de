#!/bin/bash
# round 6: H = 128 epilogue store variants: window A/B, then WRITE_SIZE / FETCH_SIZE per variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
WB_H=128 AB_OUT=gpurun_out/r6_ab_st.json bash scripts/gpu_r6_ab.sh || exit 1
for v in "" ${ST_VARIANTS:-}; do
  if [ -n "$v" ]; then export MIGNN_LIB_VARIANT=variants/libmignn_$v.so; else unset MIGNN_LIB_VARIANT; fi
  KP_H=128 KP_KINDS=win KP_REPS=2 KP_GROUPS="FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" bash scripts/gpu_kpmc.sh > /dev/null
  python scripts/kpmc_report.py gpurun_out/kpmc > gpurun_out/r6_kpmc_st_${v:-product}.json
  rm -rf gpurun_out/kpmc
  python - "gpurun_out/r6_kpmc_st_${v:-product}.json" "${v:-product}" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, c in d.items():
    print(sys.argv[2], k, "read GB", round(2 * c.get("FETCH_SIZE", 0) * 1024 / 1e9, 3),
          "write GB", round(c.get("WRITE_SIZE", 0) * 1024 / 1e9, 3))
PY
done

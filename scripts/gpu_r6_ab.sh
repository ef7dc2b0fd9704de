#!/bin/bash
# same-box A/B of window-kernel variants (WB_LIBS), optional H = 128 timeline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
out=${AB_OUT:-gpurun_out/r6_ab.json}
WB_OLD=0 WB_H=${WB_H:-128,64} WB_REPS=${WB_REPS:-7} WB_MODES=${WB_MODES:-} WB_LIBS=$WB_LIBS \
    timeout -k 10 600 python -u scripts/win_bench.py > $out 2> gpurun_out/r6_ab.err \
    || { tail -20 gpurun_out/r6_ab.err; exit 1; }
python - "$out" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for h, v in d["by_h"].items():
    print(h, {k: v["ms"][k] for k in v["ms"]}, {k: v[k] for k in v if "bitwise" in k})
PY
if [ -n "${AB_TRACE:-}" ]; then
  WT_H=128 WT_MODE=0 timeout -k 10 200 python -u scripts/win_trace.py 2> gpurun_out/wtrace.err | tee gpurun_out/r6_ab_trace.json
fi

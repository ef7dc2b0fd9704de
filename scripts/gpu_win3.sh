#!/bin/bash
# window kernel: timing study + PMC passes (win vs pc at H=128, win at H=64)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
WB_MODES=${WB_MODES:-4} timeout -k 10 400 python -u scripts/win_bench.py \
    > gpurun_out/win_bench.json 2> gpurun_out/win_bench.err || { tail -20 gpurun_out/win_bench.err; exit 1; }
cat gpurun_out/win_bench.json
rm -rf gpurun_out/kpmc
KP_KINDS=win,pc KP_H=128 bash scripts/gpu_kpmc.sh || exit 1
python scripts/kpmc_report.py gpurun_out/kpmc > gpurun_out/kpmc_win128.json && cat gpurun_out/kpmc_win128.json
rm -rf gpurun_out/kpmc
KP_KINDS=win,winagg KP_H=64 bash scripts/gpu_kpmc.sh || exit 1
python scripts/kpmc_report.py gpurun_out/kpmc > gpurun_out/kpmc_win64.json && cat gpurun_out/kpmc_win64.json

#!/bin/bash
# leg A/B: the product build against variants/libmignn_$V.so (AB_VARIANTS) on
# the bench legs named by AB_LEGS, alternating rounds (per-layer ms and ms per forward)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for round in 1 2; do
  for v in product ${AB_VARIANTS:-}; do
    if [ "$v" = product ]; then unset MIGNN_LIB_VARIANT; else export MIGNN_LIB_VARIANT=variants/libmignn_$v.so; fi
    timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu --no-bfs --no-train --no-graph --no-config4 \
        --legs "${AB_LEGS:-gat}" > gpurun_out/legab.json 2> gpurun_out/legab.err || exit $?
    echo "$v $(python -c "
import json
d = json.load(open('gpurun_out/legab.json'))
print({k: (v['ms_per_forward'], (v.get('roofline') or {}).get('avg_layer_ms')) for k, v in d['legs'].items()})")"
  done
done

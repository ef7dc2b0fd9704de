#!/bin/bash
# headline A/B: the product build against variants/libmignn_$V.so (AB_VARIANTS),
# row codes on and off, alternating rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for round in 1 2; do
  for v in product ${AB_VARIANTS:-}; do
    for c in ${AB_CODES:-1 0}; do
      if [ "$v" = product ]; then unset MIGNN_LIB_VARIANT; else export MIGNN_LIB_VARIANT=variants/libmignn_$v.so; fi
      MIGNN_GCN_CODES=$c timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-bfs --no-train --no-legs --no-config4 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
      echo "$v codes=$c $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(round(d['ms_per_step'],3),round(d['ms_per_step_graph_cached'],3),d['roofline']['avg_launch_ms'],d['roofline'].get('layers01_codes',{}).get('avg_ms'))")"
    done
  done
done

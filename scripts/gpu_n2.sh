#!/bin/bash
# rehearsal of the bench's N = 2 path on a one-GPU box (two ranks on one GPU:
# exercises the RCCL halo, the shard layout and the column-order shards; the
# timing is not a scaling number -- two processes time-slice the GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --oversubscribe --steps 3 --warmup 1 --no-cpu --no-bfs \
    --no-train --no-legs --no-config4 > gpurun_out/n2.json 2> gpurun_out/n2.err
rc=$?; echo "rc=$rc"; tail -3 gpurun_out/n2.err; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d = json.loads(open("gpurun_out/n2.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["ms_per_step_graph_cached"], d["config"]["internal_node_order"][:70])
print((d.get("roofline") or {}).get("kernel"), (d.get("roofline") or {}).get("layers01_codes"))
PY

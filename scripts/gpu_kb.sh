#!/bin/bash
# hot-kernel ablations + trace (scripts/kbench.py), GEMM parity, leg timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gemm_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
KB_ONLY=gcn16_full,gcn16_no_produce,gcn16_no_ext,gcn16_no_local,gcn16_chunks,gcn16_only_dma,copy,head16,layer0 KB_TRACE=1 \
  timeout -k 10 300 python -u scripts/kbench.py > gpurun_out/kb_r02.json 2> gpurun_out/kb_r02.err
rc=$?; cat gpurun_out/kb_r02.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/kb_r02.err; exit $rc; fi
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-bfs --no-train --no-graph --legs transformer,gin,gat > gpurun_out/bench_legs.log 2>&1
rc=$?; tail -1 gpurun_out/bench_legs.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print({k:(v['ms_per_forward'],v['roofline'].get('frac')) for k,v in d['legs'].items()})"
exit $rc

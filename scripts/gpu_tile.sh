#!/bin/bash
# round 4 hot kernel: tile-plan GCN tests, then timings (scripts/tile_bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_tile.py -k "${TILE_K:-}" > gpurun_out/tile_tests.log 2>&1
rc=$?; tail -25 gpurun_out/tile_tests.log; [ $rc -ne 0 ] && exit $rc
TB_MODES=${TB_MODES:-} TB_RING_MODES=${TB_RING_MODES:-} timeout -k 10 300 python -u scripts/tile_bench.py > gpurun_out/tile_bench.json 2> gpurun_out/tile_bench.err
rc=$?; cat gpurun_out/tile_bench.json; tail -5 gpurun_out/tile_bench.err; exit $rc

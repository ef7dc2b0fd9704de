set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -15
if [ $rc -ne 0 ]; then tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu > gpurun_out/bench.log 2>&1
rc=$?; tail -2 gpurun_out/bench.log; exit $rc

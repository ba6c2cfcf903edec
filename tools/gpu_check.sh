#!/bin/bash
# One GPU-box session: smoke -> parity tests -> bench. Every GPU step has its own time
# limit; a fault/abort/timeout (exit >= 124 or signal) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 ${SMOKE_T:-240} python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi  # a failing smoke may be a device fault: run nothing else
timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if fatal $rc || grep -q "DEVICE_FAULT\|illegal memory" gpurun_out/pytest_gpu.log; then exit 1; fi
if [ -n "$NO_BENCH" ]; then exit 0; fi
timeout -k 10 ${BENCH_T:-400} python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc

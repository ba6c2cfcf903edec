#!/bin/bash
# On the GPU box: GPU parity tests of the working tree, then same-box A/B benches of the
# default build against tools/diag_libs variants (tools/sweep.sh). usage: VARIANTS="base" tools/ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_ab.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/sweep.sh

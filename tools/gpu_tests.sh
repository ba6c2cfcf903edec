#!/bin/bash
# GPU tests only (optionally a -k expression), each with its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_sel.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_sel.log; exit $rc

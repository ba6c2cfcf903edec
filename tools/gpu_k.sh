#!/bin/bash
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_k.log; exit $rc

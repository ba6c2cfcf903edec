#!/bin/bash
# Round-6 session 18: the solo march in the plain transport_kernel (soloall) vs base on M5, M0 (LEAN=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_soloall.so PYTEST_K="skin or detectors or scat_test or validation" bash tools/gpu_tests.sh || exit 1
AB="base lib:soloall" ROUNDS=3 STEPS=10 WL=m5 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

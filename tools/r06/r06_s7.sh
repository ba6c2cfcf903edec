#!/bin/bash
# Round-6 session 7: pipelined walker emit (variant pipe) on top of the start cells (base).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_pipe.so PYTEST_K="lean or single_sphere or scat_test or refracting or deposit or bucket" bash tools/gpu_tests.sh || exit 1
AB="base lib:pipe" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:pipe" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 8: two segments per walker lane (w2d1: one crossing each per iteration,
# w2d2: two), parity on the lean path, then same-box A/B on M1 and M0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_w2d1.so PYTEST_K="lean or single_sphere or scat_test or refracting or deposit or bucket" bash tools/gpu_tests.sh || exit 1
AB="base lib:w2d1 lib:w2d2" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:w2d1 lib:w2d2" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:w2d1 lib:w2d2" ROUNDS=1 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
# the upper bound of a cheaper square root on the EVAL-bound workloads (rawsqrt: NOT exact)
AB="base lib:rawsqrt" ROUNDS=1 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:rawsqrt" ROUNDS=1 STEPS=4 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

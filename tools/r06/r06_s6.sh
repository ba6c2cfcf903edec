#!/bin/bash
# Round-6 session 6: the walker's start cells from the photon (variant sc1): lean-path parity
# tests on the variant, then same-box A/B on M1, M3, M0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_sc1.so PYTEST_K="lean or single_sphere or scat_test or refracting or deposit" bash tools/gpu_tests.sh || exit 1
AB="base lib:sc1" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:sc1" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:sc1" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

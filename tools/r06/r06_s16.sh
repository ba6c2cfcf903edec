#!/bin/bash
# Round-6 session 16: EVAL pairs (two top-level spheres/boxes as straight-line code): parity on
# the variant, A/B on M1, M0, M3, M5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_pairs.so PYTEST_K="lean or single_sphere or scat_test or refracting or skin or detectors or validation or survival or moments" bash tools/gpu_tests.sh || exit 1
AB="base lib:pairs" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:pairs" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:pairs" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:pairs" ROUNDS=2 STEPS=10 WL=m5 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

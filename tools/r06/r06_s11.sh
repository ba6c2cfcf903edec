#!/bin/bash
# Round-6 session 11: culled unroll factor on M2 (base = 2, u1, u4), parity with u4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_u4.so PYTEST_K="sphere_scene or tail_machinery or culled" bash tools/gpu_tests.sh || exit 1
PYTEST_K="sphere_scene or tail_machinery or culled" bash tools/gpu_tests.sh || exit 1
AB="base lib:u4 lib:u1" ROUNDS=3 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

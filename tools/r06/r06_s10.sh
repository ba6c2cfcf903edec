#!/bin/bash
# Round-6 session 10: culled EVAL two spheres at a time (u2) vs base: parity on the culled
# scenes with the variant, then A/B on M2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_u2.so PYTEST_K="sphere_scene or tail_machinery or far_field or culled or nested or many_tops" bash tools/gpu_tests.sh || exit 1
AB="base lib:u2 lib:noctab" ROUNDS=3 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

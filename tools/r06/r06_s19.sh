#!/bin/bash
# Round-6 session 19: pairs in the event waves' reflect_refract EVALs (evpairs) vs base on M3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_evpairs.so PYTEST_K="lean_kernel_paths or refracting or modifier_scenes" bash tools/gpu_tests.sh || exit 1
AB="base lib:evpairs" ROUNDS=3 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

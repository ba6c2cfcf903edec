#!/bin/bash
# Round-6 session 37: the plain ws_kernel with the deferral box from KParams (kbp) against base (VGPR
# box), now that the plain unit schedules with the AMDGPU trackers; M1, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="lean or scat_test or single_sphere" SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_kbp.so bash tools/gpu_tests.sh || exit 1
AB="base lib:kbp" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

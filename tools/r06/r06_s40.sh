#!/bin/bash
# Round-6 session 40: the photon waves read their busy bits once per trip (base) vs at each check
# (bs0): the lean-path GPU tests on base, then same-box A/B on M1 and M3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="lean or scat_test or single_sphere or refracting or watchdog or deposit or bucket or spectral or fortran" bash tools/gpu_tests.sh || exit 1
AB="base lib:bs0" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:bs0" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

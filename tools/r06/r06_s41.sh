#!/bin/bash
# Round-6 session 41: a walker frees a segment slot right after the crossing that ends it (base) vs after the
# iteration's last crossing (ef0): the lean-path GPU tests on base, then same-box A/B on M1 and M3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="lean or scat_test or single_sphere or refracting or watchdog or deposit or bucket or spectral or fortran" bash tools/gpu_tests.sh || exit 1
AB="base lib:ef0" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:ef0" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

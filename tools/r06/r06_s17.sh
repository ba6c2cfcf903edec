#!/bin/bash
# Round-6 session 17: EVAL pairs in transport_kernel only (base) vs none (nopairs): the GPU suite
# subset for transport_kernel scenes, A/B on M5 and M1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
PYTEST_K="not lean_kernel_paths and not watchdog and not fortran" bash tools/gpu_tests.sh || exit 1
AB="base lib:nopairs" ROUNDS=3 STEPS=10 WL=m5 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:nopairs" ROUNDS=2 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

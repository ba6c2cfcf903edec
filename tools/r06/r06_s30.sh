#!/bin/bash
# Round-6 session 30: capture EVALs of culled scenes fold only the captured tops (base) vs a full
# EVAL of every top (cap0): culled/Fresnel GPU tests on base, then same-box A/B on M2 and M4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="sphere_scene or culled or vessels or far_ or coop or many_tops or nested or modifier or tail_machinery or skin or fresnel or refract" bash tools/gpu_tests.sh || exit 1
AB="base lib:cap0" ROUNDS=3 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:cap0" ROUNDS=2 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

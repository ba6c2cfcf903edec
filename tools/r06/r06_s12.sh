#!/bin/bash
# Round-6 session 12: the unrolled culled EVAL for spheres and capsules (base, U = 4) vs none
# (u1): parity on the culled scenes incl. M4's vessels, then A/B on M4 and M2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
PYTEST_K="sphere_scene or tail_machinery or culled or vessel or far or many_tops or nested or egg or modifier" bash tools/gpu_tests.sh || exit 1
AB="base lib:u1" ROUNDS=2 STEPS=4 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:u1" ROUNDS=2 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 14: culled groups by list flags (base: spheres from the table, capsules from
# nodes, U = 4) vs the committed sphere-only unroll (prev) and U = 2 (cap2): parity, M4, M2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
PYTEST_K="sphere_scene or tail_machinery or culled or vessel or far or many_tops or nested or egg or modifier" bash tools/gpu_tests.sh || exit 1
AB="base lib:prev lib:cap2" ROUNDS=2 STEPS=4 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:prev lib:cap2" ROUNDS=2 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 15: spheres by 4 + capsules by 2 (base) vs the committed sphere-only unroll
# (prev) and both by 2 (cap2): parity, M4, M2 (three rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
PYTEST_K="sphere_scene or tail_machinery or culled or vessel or far or many_tops or nested" bash tools/gpu_tests.sh || exit 1
AB="base lib:prev lib:cap2" ROUNDS=3 STEPS=4 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:prev lib:cap2" ROUNDS=3 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

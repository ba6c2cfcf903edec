#!/bin/bash
# Round-6 session 9: the culled EVAL reading listed tops from the LDS table (base) vs device
# memory (noctab): GPU parity of the culled scenes, then A/B on M2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
PYTEST_K="sphere_scene or tail_machinery or far_field or culled or nested or many_tops or general_emitter" bash tools/gpu_tests.sh || exit 1
AB="base lib:noctab" ROUNDS=2 STEPS=4 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

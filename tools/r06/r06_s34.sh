#!/bin/bash
# Round-6 session 34: capsules divide with a per-scene reciprocal in P(7) (base) vs in full (crcp0):
# capsule/culled GPU tests on base, then same-box A/B on M4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="vessels or culled or coop or many_tops or nested or modifier or far_ or classify or escape or sphere_scene or general_emitter" bash tools/gpu_tests.sh || exit 1
AB="base lib:crcp0" ROUNDS=3 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

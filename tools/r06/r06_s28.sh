#!/bin/bash
# Round-6 session 28: culled lists nearest box first with per-entry bounds; a lane stops its list
# walk once the rest is farther than its min|ds| (base) vs the same lists walked to the end (elb0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="sphere_scene or culled or vessels or far_ or coop or many_tops or nested or modifier or tail_machinery or skin" bash tools/gpu_tests.sh || exit 1
AB="base lib:elb0" ROUNDS=3 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:elb0" ROUNDS=2 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

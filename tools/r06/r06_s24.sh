#!/bin/bash
# Round-6 session 24: the split kinst units (plain ws_kernel with the AMDGPU trackers): the whole
# GPU suite, M1 and M3 lines, then the culling list-rule A/B (r06_s23.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
AB="base" ROUNDS=2 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base" ROUNDS=1 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
bash tools/r06/r06_s23.sh

#!/bin/bash
# Round-6 session 43: scheduler flags for transport_kernel (M2, M4, M5): the whole library with the
# AMDGPU trackers (trk) or max-ilp (ilp) against base (part 0 with the default scheduler).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base lib:trk lib:ilp" ROUNDS=2 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:trk lib:ilp" ROUNDS=2 STEPS=10 WL=m5 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:trk lib:ilp" ROUNDS=2 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

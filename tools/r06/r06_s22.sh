#!/bin/bash
# Round-6 session 22: AMDGPU scheduler strategies for the whole library (ilp: max-ilp, trk: the
# AMDGPU register-pressure trackers, mem: max-memory-clause) against base, same box, M1 and M3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base lib:ilp lib:trk lib:mem" ROUNDS=2 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:ilp lib:trk lib:mem" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 36 (second pass: 16, 24, 40; first pass: 6, 3, 1): the sparse-wave threshold of the cooperative table EVAL on culled M2
# (SMCRT_COOP_LANES; default n_top / 4 = 10 for 41 tops), 6 steps, same box; then M4 (3 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base env:SMCRT_COOP_LANES=16 env:SMCRT_COOP_LANES=24 env:SMCRT_COOP_LANES=40" ROUNDS=2 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1


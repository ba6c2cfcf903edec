#!/bin/bash
# Round-6 session 42: the cooperative table EVAL's sparse-wave threshold on M2 once more
# (SMCRT_COOP_LANES 12 and 16 vs the default 10), 3 rounds of 6 steps, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base env:SMCRT_COOP_LANES=12 env:SMCRT_COOP_LANES=16" ROUNDS=3 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

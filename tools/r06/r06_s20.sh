#!/bin/bash
# Round-6 session 20: the event waves' straight-line interaction (base, SMCRT_WS_EV_SL=1) against
# the branchy one (evsl0): the whole GPU suite on base, then same-box A/B on M1 and M3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
AB="base lib:evsl0" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:evsl0" ROUNDS=2 STEPS=10 WL=m3 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

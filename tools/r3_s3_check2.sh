#!/bin/bash
# Round-3 session-3 check 2: smoke, parity tests (nested models), bench, slot A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh || exit 1
WL=m1 STEPS=10 ENVS="SMCRT_SLOTS=4" bash tools/exp_env.sh | sed "s/^/m1 /" || exit 1
WL=m1 STEPS=10 ENVS="SMCRT_SLOTS=4" bash tools/exp_env.sh | sed "s/^/m1 /" || exit 1
WL=m2 STEPS=3 ENVS="SMCRT_SLOTS=2" bash tools/exp_env.sh | sed "s/^/m2 /" || exit 1

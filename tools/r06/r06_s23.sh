#!/bin/bash
# Round-6 session 23: the culling grid's list rule on the culled workloads (M2: 40 spheres, M4: 512
# capsules): K nearest tops per cell (SMCRT_CULL_K, default 8) and cells per top (SMCRT_CULL_CPT,
# default 64). Exact either way (the device's bound test falls back to the full EVAL).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base env:SMCRT_CULL_K=4 env:SMCRT_CULL_K=2 env:SMCRT_CULL_CPT=512 env:SMCRT_CULL_CPT=512,env:SMCRT_CULL_K=3" ROUNDS=2 STEPS=3 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base env:SMCRT_CULL_K=4 env:SMCRT_CULL_K=2 env:SMCRT_CULL_CPT=256,env:SMCRT_CULL_K=4" ROUNDS=2 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 25: the culling grid's list rule, second pass: the reach U scaled down
# (SMCRT_CULL_UFRAC; 0 = the K nearest only) and finer grids (SMCRT_CULL_CPT), on M2 and M4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base env:SMCRT_CULL_CPT=512 env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=2 env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=3 env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=4 env:SMCRT_CULL_UFRAC=0.5 env:SMCRT_CULL_CPT=512,env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=3 env:SMCRT_CULL_CPT=2048,env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=3" ROUNDS=2 STEPS=3 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base env:SMCRT_CULL_CPT=256 env:SMCRT_CULL_CPT=512 env:SMCRT_CULL_CPT=256,env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=4 env:SMCRT_CULL_CPT=256,env:SMCRT_CULL_UFRAC=0.5 env:SMCRT_CULL_CPT=512,env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=3" ROUNDS=2 STEPS=3 WL=m4 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 27: more AMDGPU scheduler strategies on top of the split units (base = the
# trackers for the plain ws_kernel): iterative-ilp, iterative-maxocc, iterative-minreg, metric bias 100.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base lib:itilp lib:itocc lib:itmin lib:bias100" ROUNDS=2 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

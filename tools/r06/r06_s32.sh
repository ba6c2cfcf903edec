#!/bin/bash
# Round-6 session 32: M5 (detectors + Fresnel) on transport_kernel (base) vs the XF lean path now
# that its scratch fell to 116 B (SMCRT_LEAN=1), 10 steps, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base env:SMCRT_LEAN=1" ROUNDS=2 STEPS=10 WL=m5 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

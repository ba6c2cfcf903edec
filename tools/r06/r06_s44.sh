#!/bin/bash
# Round-6 session 44: three crossings per walker iteration (dda3) against two (base) under the
# trackers scheduler, M1 and M0 (8 crossings per segment), same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
AB="base lib:dda3" ROUNDS=2 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:dda3" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

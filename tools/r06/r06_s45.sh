#!/bin/bash
# Round-6 session 45: a point source's emission carries the layer (the layer search at the source
# point, formed once per launch) and the first tauint2 entry (base) vs separate events (et0):
# the whole GPU suite on base, then same-box A/B on M1, M0 (point sources) and M3 (line source).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit 1
AB="base lib:et0" ROUNDS=3 STEPS=10 WL=m1 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
AB="base lib:et0" ROUNDS=2 STEPS=10 WL=m0 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

#!/bin/bash
# Round-6 session 5: tail priority A/B on the tail-bound workloads and M1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
for wl in m5 m4 m2 m1; do
  st=10; [ $wl = m2 ] && st=4; [ $wl = m4 ] && st=4
  AB="base lib:tail8 lib:tail16p1" ROUNDS=2 STEPS=$st WL=$wl bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1
done

#!/bin/bash
# Round-3 session-3: GPU tests on the nested-model build, then same-box A/B against the build
# before nested models (tools/diag_libs/libsmcrt_prenest.so = d5b0c73) on the non-lean scenes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
NO_BENCH=1 bash tools/gpu_check.sh || exit 1
for wl in m5 m3 m0 m4 m1; do
  st=3; [ $wl = m4 ] && st=2; [ $wl = m1 ] && st=10
  AB_WORKLOAD=$wl AB_LIBS="base prenest" BENCH_ARGS="--steps $st" bash tools/ab_libs.sh | sed "s/^/$wl /" || exit 1
done

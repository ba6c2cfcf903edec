#!/bin/bash
# Round-3 session-3: GPU tests on the nested-model build, then same-box A/B against the build
# before nested models (tools/diag_libs/libsmcrt_prenest.so = d5b0c73) on the non-lean scenes,
# and of the cull-list prefetch (nopf = -DSMCRT_CULL_PREFETCH=0) on M4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
NO_BENCH=1 bash tools/gpu_check.sh || exit 1
for wl in m4 m5 m3 m0 m1; do
  st=3; libs="base prenest"; [ $wl = m4 ] && { st=2; libs="base prenest nopf"; }; [ $wl = m1 ] && st=10
  AB_WORKLOAD=$wl AB_LIBS="$libs" BENCH_ARGS="--steps $st" bash tools/ab_libs.sh | sed "s/^/$wl /" || exit 1
done

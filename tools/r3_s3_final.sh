#!/bin/bash
# Round-3 session-3 final check at HEAD: smoke, GPU tests, bench; then the non-lean scenes
# against the build before nested models (tools/diag_libs/libsmcrt_prenest.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh || exit 1
for wl in m5 m0 m3; do
  AB_WORKLOAD=$wl AB_LIBS="base prenest" BENCH_ARGS="--steps 3" bash tools/ab_libs.sh | sed "s/^/$wl /" || exit 1
done

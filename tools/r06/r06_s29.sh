#!/bin/bash
# Round-6 session 29: diagnostic build (-DSMCRT_DIAG) on M2, M4 and M1: phase shares and the
# culled EVAL's statistics (list entries walked, bound-test fallbacks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in ${WLS:-m2 m4 m1}; do
  SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so timeout -k 10 300 python bench.py --workload $wl --steps 2 --warmup 1 --no-cpu --no-ref > gpurun_out/diag_$wl.json 2> gpurun_out/diag_$wl.err || { tail -5 gpurun_out/diag_$wl.err; exit 1; }
  echo "== $wl"; grep -h "diag" gpurun_out/diag_$wl.err | tail -8
done

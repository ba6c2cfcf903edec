#!/bin/bash
# Per-phase wave time, lane states and culling counters (-DSMCRT_DIAG build in
# tools/diag_libs/libsmcrt_diag.so) for M4, M2 and M5; output gpurun_out/diag_<w>.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so
for spec in ${DIAG_RUNS:-"m4:1000000 m2:100000 m5:4000000"}; do
  w=${spec%%:*}; n=${spec##*:}
  timeout -k 10 240 python3 tools/diag_phases.py $n $w > gpurun_out/diag_$w.txt 2>&1 || { echo "$w failed"; tail -5 gpurun_out/diag_$w.txt; exit 1; }
  echo "== $w"; grep -v "amdgpu.ids" gpurun_out/diag_$w.txt | tail -12
done

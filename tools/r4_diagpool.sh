#!/bin/bash
# Round 4: -DSMCRT_DIAG schedule tallies of the lean kernel with and without the event pool (M1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_diagpool
for v in diagnopool diagpool; do
  SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so timeout -k 10 240 python3 tools/diag_phases.py 16000000 m1 > gpurun_out/r04_diagpool/$v.txt 2>&1 || { tail -5 gpurun_out/r04_diagpool/$v.txt; exit 1; }
  echo "== $v"; grep -E "diag-lean|diag-time" gpurun_out/r04_diagpool/$v.txt | tail -2
done

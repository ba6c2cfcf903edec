#!/bin/bash
# Round-6 session 3: phase shares (diag library) of M2 and M5, slowest photons of M5 and M2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tail gpurun_out/phases
export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so
for w in m2:4000000 m5:3000000 m4:2000000; do
  timeout -k 10 240 python -u tools/diag_phases.py ${w##*:} ${w%%:*} > gpurun_out/phases/${w%%:*}.txt 2>&1 || { tail -20 gpurun_out/phases/${w%%:*}.txt; exit 1; }
  echo "== phases ${w%%:*}"; grep -v "^\[diag\]" gpurun_out/phases/${w%%:*}.txt | tail -14
done
for w in m5:6000000 m2:12800000; do
  SMCRT_DIAG_DONE=1 timeout -k 10 300 python -u tools/tail_profile.py ${w%%:*} ${w##*:} gpurun_out/tail/${w%%:*}_ids.json > gpurun_out/tail/${w%%:*}_ids.txt 2>&1 || { tail -20 gpurun_out/tail/${w%%:*}_ids.txt; exit 1; }
  echo "== tail ${w%%:*}"; grep "slowest\|share_after" -A3 gpurun_out/tail/${w%%:*}_ids.txt | head -12
done

#!/bin/bash
# Round-6 session 2: per-photon completion profiles (diag library) of the tail-bound workloads,
# then whether rocprofv3 PC sampling works on this box (list + a short run's first lines).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tail
for w in m2:25600000 m4:8000000 m5:6000000 m1:16000000; do
  SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so SMCRT_DIAG_DONE=1 timeout -k 10 300 \
    python -u tools/tail_profile.py ${w%%:*} ${w##*:} gpurun_out/tail/${w%%:*}.json > gpurun_out/tail/${w%%:*}.txt 2>&1 || { tail -20 gpurun_out/tail/${w%%:*}.txt; exit 1; }
  echo "== ${w%%:*}"; grep -v "^\[" gpurun_out/tail/${w%%:*}.txt | head -40
done
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/rocprof_list.txt 2>&1
grep -i -A20 "pc.sampl\|PC_SAMPL" $GRAFT_REPO_ROOT/gpurun_out/rocprof_list.txt | head -60

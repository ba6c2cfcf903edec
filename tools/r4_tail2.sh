#!/bin/bash
# Round 4: lane states of M4's tail (waves with <= 4 photons left), -DSMCRT_DIAG_STATES -DSMCRT_DIAG_TAIL.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r04_tail; mkdir -p $out
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_tail.so timeout -k 10 240 python3 tools/diag_phases.py 8000000 m4 > $out/tail_states_m4.txt 2>&1 || { tail -5 $out/tail_states_m4.txt; exit 1; }
grep -v amdgpu.ids $out/tail_states_m4.txt | tail -8

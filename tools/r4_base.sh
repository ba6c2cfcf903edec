#!/bin/bash
# Round-4 baseline on a fresh box: smoke, GPU tests, bench at HEAD, then the lean kernel's
# -DSMCRT_DIAG schedule tallies and phase shares on M1 (tools/diag_libs/libsmcrt_diag.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/r04_base
cp gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench.json gpurun_out/r04_base/
SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so timeout -k 10 240 python3 tools/diag_phases.py 16000000 m1 > gpurun_out/r04_base/diag_m1.txt 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/r04_base/diag_m1.txt | tail -12; exit $rc

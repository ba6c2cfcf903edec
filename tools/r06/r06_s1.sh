#!/bin/bash
# Round-6 session 1 on the GPU box: the new tests, the whole GPU suite, the bench, then a same-box
# A/B of the inline-event variants and the M1 diag breakdown.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTEST_K="watchdog or spectral" bash tools/gpu_tests.sh || exit 1
bash tools/base_r06.sh || exit 1
AB="base lib:inl32 lib:inl96 lib:inl192" ROUNDS=2 WL=m1 bash tools/ab.sh > gpurun_out/ab_inline.txt 2>&1 || { cat gpurun_out/ab_inline.txt; exit 1; }
cat gpurun_out/ab_inline.txt
AB="lib:diag" ROUNDS=1 STEPS=2 WL=m1 bash tools/ab.sh > /dev/null 2>&1
grep -h "diag-ws" gpurun_out/ab/m1_lib_diag.err | tail -2

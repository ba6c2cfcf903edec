#!/bin/bash
# Round 4 session 1: the new parity tests (modifiers, egg, nested models, lean hazards, far
# field), then M1 A/B of the in-tree build against 4 waves/SIMD with two lean slots.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_s1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "egg or modifier or nested or hazard or far_field or single_sphere" > gpurun_out/r04_s1/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r04_s1/pytest.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=m1 AB_LIBS="base w4s2" BENCH_ARGS="--steps 10" bash tools/ab_libs.sh | tee gpurun_out/r04_s1/ab_w4s2.txt

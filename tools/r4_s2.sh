#!/bin/bash
# Round 4 session 2: culled EVAL with LDS primitive records (M4) parity + env A/B, then the
# event-pool A/B (tools/r4_pool.sh's libraries) on M1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_s2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "cull or vessel or tail or many or mixed or lean" > gpurun_out/r04_s2/pytest.log 2>&1
rc=$?; tail -12 gpurun_out/r04_s2/pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  WL=m4 STEPS=3 ENVS="SMCRT_CULL_LTAB=0" bash tools/exp_env.sh | tee -a gpurun_out/r04_s2/ab_m4_ltab.txt || exit 1
done
AB_WORKLOAD=m1 AB_LIBS="base nopool loc4 p32" BENCH_ARGS="--steps 10" bash tools/ab_libs.sh | tee gpurun_out/r04_s2/ab_pool.txt

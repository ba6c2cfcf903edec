#!/bin/bash
# Round 4: the lean kernel's block event pool. Parity first (lean paths, hazards, M1, smoke),
# then M1 A/B: in-tree (pool, 48) against no pool and pool thresholds 32 / 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r04_pool
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_pool/smoke.log 2>&1 || { cat gpurun_out/r04_pool/smoke.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "lean or hazard or single_sphere or scat_test or bucket or absorb" > gpurun_out/r04_pool/pytest.log 2>&1
rc=$?; tail -15 gpurun_out/r04_pool/pytest.log; [ $rc -ne 0 ] && exit $rc
AB_WORKLOAD=m1 AB_LIBS="base nopool loc4 p32" BENCH_ARGS="--steps 10" bash tools/ab_libs.sh | tee gpurun_out/r04_pool/ab.txt

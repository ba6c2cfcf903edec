#!/bin/bash
# On the GPU box: bench each tools/diag_libs/libsmcrt_<name>.so (and the default build).
# usage: VARIANTS="a b c" tools/sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in default $VARIANTS; do
  if [ $v = default ]; then unset SMCRT_LIB; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  timeout -k 10 240 python bench.py --no-cpu --steps ${STEPS:-5} --warmup 2 ${BENCH_EXTRA} > gpurun_out/sweep_$v.json 2> gpurun_out/sweep_$v.err
  rc=$?; if [ $rc -ne 0 ]; then echo "$v rc=$rc"; tail -5 gpurun_out/sweep_$v.err; exit $rc; fi
  python3 -c "import json;d=json.load(open('gpurun_out/sweep_$v.json'));r=d['roofline'];print('%-12s %.4e ph/s  transport %.2f ms  fold %.2f ms  iters %.3g' % ('$v', d['value'], r['avg_launch_ms'], r['deposit_fold_ms_per_launch'], r['wave_iterations_per_launch']))"
done

#!/bin/bash
# Same-box A/B of a bench.py workload: the working-tree library against tools/diag_libs
# variants. usage: WL=m4 VARIANTS="head" [BATCH=..] [STEPS=3] tools/exp_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in new $VARIANTS; do
  if [ $v = new ]; then unset SMCRT_LIB; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  timeout -k 10 ${AB_T:-300} python3 bench.py --workload ${WL:-m1} ${BATCH:+--batch $BATCH} --steps ${STEPS:-3} --warmup 1 \
    --no-cpu --no-ref ${AB_EXTRA} > gpurun_out/ab_${WL:-m1}_$v.json 2> gpurun_out/ab_${WL:-m1}_$v.err || { echo "$v failed"; tail -3 gpurun_out/ab_${WL:-m1}_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_${WL:-m1}_$v.json'));r=d['roofline'];print('${WL:-m1} %-6s %.4e ph/s  ms/step %.1f  transport %.1f ms  fold_cu %.2f ms  iters %.4g' % ('$v', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('fold_cu_ms_per_launch', 0), r['wave_iterations_per_launch']))"
done

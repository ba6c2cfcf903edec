#!/bin/bash
# Same-box A/B over (library, environment) pairs for one bench.py workload.
# usage: WL=m1 RUNS="new: t12:SMCRT_LEAN_SPARE=32 ..." [STEPS=..] tools/exp_matrix.sh
#   "lib:A=1,B=2" -- lib "new" is the working tree, else tools/diag_libs/libsmcrt_<lib>.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
i=0
for run in $RUNS; do
  i=$((i+1)); lib=${run%%:*}; envs=${run#*:}
  ( if [ $lib != new ]; then export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$lib.so; fi
    [ -n "$envs" ] && for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 ${AB_T:-300} python3 bench.py --workload ${WL:-m1} ${BATCH:+--batch $BATCH} --steps ${STEPS:-3} --warmup 1 \
      --no-cpu --no-ref ${AB_EXTRA} > gpurun_out/mx_$i.json 2> gpurun_out/mx_$i.err ) || { echo "$run failed"; tail -3 gpurun_out/mx_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/mx_$i.json'));r=d['roofline'];print('%-40s %.4e ph/s  ms/step %.1f  transport %.1f ms  fold_cu %.2f' % ('$run', d['value'], d['ms_per_step'], r['avg_launch_ms'], r.get('fold_cu_ms_per_launch', 0)))"
done

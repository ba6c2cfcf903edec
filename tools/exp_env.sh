#!/bin/bash
# Same-box sweep of environment settings for one bench.py workload.
# usage: WL=m4 ENVS="A=1,B=2 A=3" [STEPS=3] [BATCH=..] tools/exp_env.sh  (',' separates variables)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
i=0
for e in default $ENVS; do
  i=$((i+1))
  ( [ $e != default ] && for kv in ${e//,/ }; do export "$kv"; done
    timeout -k 10 ${AB_T:-300} python3 bench.py --workload ${WL:-m1} ${BATCH:+--batch $BATCH} --steps ${STEPS:-3} --warmup 1 \
      --no-cpu --no-ref ${AB_EXTRA} > gpurun_out/env_$i.json 2> gpurun_out/env_$i.err ) || { echo "$e failed"; tail -3 gpurun_out/env_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/env_$i.json'));r=d['roofline'];print('%-50s %.4e ph/s  ms/step %.1f  transport %.1f ms  iters %.4g' % ('$e', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['wave_iterations_per_launch']))"
done

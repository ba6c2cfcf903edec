#!/bin/bash
# M2 A/B: the cooperative EVAL from the LDS table (default) against SMCRT_COOP_TAB=0.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
B=${M2_BATCH:-400000}
for v in tab notab; do
  if [ $v = notab ]; then export SMCRT_COOP_TAB=0; else unset SMCRT_COOP_TAB; fi
  timeout -k 10 300 python3 bench.py --workload m2 --batch $B --steps ${STEPS:-3} --warmup 1 --no-cpu --no-ref \
    > gpurun_out/m2_$v.json 2> gpurun_out/m2_$v.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/m2_$v.json'));r=d['roofline'];print('$v %.4e ph/s  ms/step %.0f  transport %.1f ms  iters %.4g' % (d['value'], d['ms_per_step'], r['avg_launch_ms'], r['wave_iterations_per_launch']))"
done

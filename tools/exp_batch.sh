#!/bin/bash
# Photons-per-step sweep of one workload (same box). usage: WL=m4 BATCHES="4000000 8000000" tools/exp_batch.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for b in $BATCHES; do
  timeout -k 10 ${AB_T:-300} python3 bench.py --workload ${WL:-m1} --batch $b --steps ${STEPS:-3} --warmup 1 --no-cpu --no-ref \
    > gpurun_out/batch_${WL}_$b.json 2> gpurun_out/batch_${WL}_$b.err || { echo "$b failed"; tail -3 gpurun_out/batch_${WL}_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/batch_${WL}_$b.json'));r=d['roofline'];print('${WL} %-9s %.4e ph/s  ms/step %.1f  transport %.1f ms x %d' % ('$b', d['value'], d['ms_per_step'], r['avg_launch_ms'], r['launches_timed']))"
done

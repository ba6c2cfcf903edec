#!/bin/bash
# Every bench.py workload once on one GPU (SURVEY §8(d) M0-M5 + escape); lines to gpurun_out/wl_<name>.json
set -e
export PYTHONUNBUFFERED=1
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in m1 m0 m2 m3 m4 m5; do
  timeout -k 10 240 python -u bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --cpu-seconds ${CPU_S:-8} --no-ref \
    > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err
  echo "$w done"
done
timeout -k 10 300 python -u bench.py --workload escape ${ESC_ARGS:-} > gpurun_out/wl_escape.json 2> gpurun_out/wl_escape.err
echo "escape done"

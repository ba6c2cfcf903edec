#!/bin/bash
# Selected bench.py workloads once on one GPU, as tools/bench_all.sh: WLS="m2 m4" tools/bench_some.sh
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for w in ${WLS:-m1}; do
  timeout -k 10 ${WL_T:-300} python -u bench.py --workload $w --steps ${STEPS:-2} --warmup 1 --cpu-seconds ${CPU_S:-8} --no-ref \
    > gpurun_out/wl_$w.json 2> gpurun_out/wl_$w.err || exit $?
  echo "$w done"
done

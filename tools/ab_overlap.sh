#!/bin/bash
# A/B of SMCRT_FLAG_OVERLAP (bench --overlap 0/1) on several workloads, one box.
# usage (GPU box): bash tools/ab_overlap.sh "m1:0 m4:1000000 m5:0"   (workload:batch, 0 = default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for wb in ${1:-"m1:0 m4:0 m5:0"}; do
  w=${wb%%:*}; b=${wb##*:}
  for ov in 0 1; do
    f=gpurun_out/ab/${w}_b${b}_ov${ov}
    timeout -k 10 300 python bench.py --workload $w --batch $b --steps ${STEPS:-4} --warmup 1 --no-cpu --no-ref \
      --overlap $ov > $f.json 2> $f.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$w ov=$ov rc=$rc"; tail -3 $f.err; exit $rc; fi
    python3 -c "import json;d=json.load(open('$f.json'));r=d['roofline'];print('$w batch=$b overlap=$ov', round(d['value']/1e6,3), 'M/s  step', round(d['ms_per_step'],1), 'ms  kernel', round(r['avg_launch_ms'],1), 'ms')"
  done
done

#!/bin/bash
# Round 4: M4/M5 tail vs bulk. -DSMCRT_DIAG phase shares and longest/mean wave ticks on one
# launch, then bench lines at 3 and 10 timed steps (no CPU leg). Output gpurun_out/r04_tail/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r04_tail; mkdir -p $out
for w in m4 m5; do
  n=8000000; [ $w = m5 ] && n=6000000
  SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so timeout -k 10 240 python3 tools/diag_phases.py $n $w > $out/diag_$w.txt 2>&1 || { tail -5 $out/diag_$w.txt; exit 1; }
  grep -v amdgpu.ids $out/diag_$w.txt | tail -14
  for s in 3 10; do
    timeout -k 10 300 python -u bench.py --workload $w --steps $s --warmup 1 --no-cpu --no-ref > $out/b_${w}_$s.json 2> $out/b_${w}_$s.err || { tail -5 $out/b_${w}_$s.err; exit 1; }
    python3 -c "import json;d=json.load(open('$out/b_${w}_$s.json'));print('$w steps $s', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],1), 'ms/step launch', round(d['roofline']['avg_launch_ms'],1))"
  done
done

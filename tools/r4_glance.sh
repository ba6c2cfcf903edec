#!/bin/bash
# Round 4: far-field glance + culled far march: targeted GPU parity tests, then M4 / M2 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
out=gpurun_out/r04_glance; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu \
  -k "far_glance or far_field_march or tail_machinery or vessels or culled" > $out/pytest.log 2>&1
rc=$?; tail -25 $out/pytest.log; [ $rc = 0 ] || exit $rc
for w in m4 m2; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-ref > $out/b_$w.json 2> $out/b_$w.err || { tail -5 $out/b_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$out/b_$w.json'));r=d['roofline'];print('$w', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],1), 'ms/step launch', round(r['avg_launch_ms'],1), 'far', r.get('far_march_steps_per_launch'))"
done

#!/bin/bash
# Round 5 A/B on one box: smoke -> selected GPU tests -> M1 bench with each SMCRT_* setting in
# $AB (space-separated NAME=VAL[,NAME=VAL] groups, "-" = defaults). Every GPU step has its own
# time limit; a fault/abort/timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/ab/smoke.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_T:-400} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTS" > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/ab/pytest.log
  if fatal $rc || [ $rc -ne 0 ]; then exit 1; fi
fi
for v in ${AB:--}; do
  envs=""; [ "$v" != "-" ] && envs=$(echo "$v" | tr ',' ' ')
  env $envs timeout -k 10 ${BENCH_T:-240} python bench.py --no-ref --cpu-seconds 4 --cpu1-seconds 0 ${BENCH_ARGS} > gpurun_out/ab/bench_$v.json 2> gpurun_out/ab/bench_$v.err
  rc=$?
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms/step, launch', round(r['avg_launch_ms'],2), 'fold_int', round(r['fold_interval_ms_per_launch'],2), 'exact', d['parity']['counters_bit_exact_vs_cpu'], d['parity']['jmean_max_rel_diff_vs_cpu'])" gpurun_out/ab/bench_$v.json "$v" || tail -5 gpurun_out/ab/bench_$v.err
  if fatal $rc || [ $rc -ne 0 ]; then exit 1; fi
done

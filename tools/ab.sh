#!/bin/bash
# Same-box A/B on the GPU box: smoke, optional GPU tests, then bench.py lines for each variant,
# ROUNDS interleaved rounds. A variant is "base" (the in-tree library), "lib:NAME"
# (tools/diag_libs/libsmcrt_NAME.so, built by tools/variants.sh) or "env:K=V[,K2=V2]" (the
# in-tree library with those variables); "lib:NAME,env:K=V" combines both.
#   AB="base lib:pw3 env:SMCRT_LEAN=0" [WL=m1] [ROUNDS=2] [STEPS=10] [TESTS="pytest -k expr"] bash tools/ab.sh
# Every GPU step has its own time limit; a fault, abort or timeout stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ab/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/ab/smoke.log; [ $rc -ne 0 ] && exit $rc
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_T:-600} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$TESTS" \
    > gpurun_out/ab/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/ab/pytest.log
  [ $rc -ne 0 ] && exit 1
fi
WL=${WL:-m1}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${AB:-base}; do
    tag=$(echo "$v" | tr ':=,/' '____')
    ( unset SMCRT_LIB
      for part in ${v//,env:/ env:}; do
        case $part in
          lib:*) export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_${part#lib:}.so ;;
          env:*) for kv in ${part#env:}; do export "$kv"; done ;;
        esac
      done
      timeout -k 10 ${BENCH_T:-240} python bench.py --workload $WL --steps ${STEPS:-10} --warmup 2 --no-cpu --no-ref \
        ${BENCH_ARGS} > gpurun_out/ab/${WL}_$tag.json 2> gpurun_out/ab/${WL}_$tag.err )
    rc=$?
    if fatal $rc || [ $rc -ne 0 ]; then echo "$v failed rc=$rc"; tail -5 gpurun_out/ab/${WL}_$tag.err; exit 1; fi
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('%-36s %7.2f M/s %6.2f ms/step  launch %6.2f  fold_int %6.2f  fold_cu %5.2f' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], r['avg_launch_ms'], r['fold_interval_ms_per_launch'], r['fold_cu_ms_per_launch']))" gpurun_out/ab/${WL}_$tag.json "$v"
  done
done

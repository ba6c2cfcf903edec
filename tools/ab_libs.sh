#!/bin/bash
# Same-box A/B of library variants (tools/diag_libs/libsmcrt_<name>.so; "base" = the in-tree
# build, "lean" = the in-tree build with SMCRT_LEAN_WS=0, "oldk" = with SMCRT_LEAN=0) on one
# workload: AB_LIBS="base s2 s4", two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
W=${AB_WORKLOAD:-m1}
for r in 1 2; do
  for v in ${AB_LIBS:-base}; do
    unset SMCRT_LEAN SMCRT_LEAN_WS
    if [ $v = base ]; then unset SMCRT_LIB
    elif [ $v = lean ]; then unset SMCRT_LIB; export SMCRT_LEAN_WS=0  # lean_kernel on the base build
    elif [ $v = oldk ]; then unset SMCRT_LIB; export SMCRT_LEAN=0  # transport_kernel on the base build
    else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
    timeout -k 10 200 python3 bench.py --workload $W --no-cpu --no-ref ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms/step', 'launch', round(d['roofline']['avg_launch_ms'],2))"
  done
done

#!/bin/bash
# Same-box A/B of the lean kernel (lean.h) against transport_kernel (SMCRT_LEAN=0) on M1, plus
# the -DSMCRT_DIAG schedule tallies of both (tools/diag_libs/libsmcrt_diag.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
W=${AB_WORKLOAD:-m1}
if [ -z "$NO_DIAG" ]; then
  SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so timeout -k 10 150 python3 tools/diag_phases.py ${DIAG_N:-4000000} $W > gpurun_out/diag_lean.txt 2>&1 || { echo diag lean failed; tail -5 gpurun_out/diag_lean.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/diag_lean.txt | tail -4
  SMCRT_LEAN=0 SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so timeout -k 10 150 python3 tools/diag_phases.py ${DIAG_N:-4000000} $W > gpurun_out/diag_old.txt 2>&1 || { echo diag old failed; exit 1; }
  grep -v amdgpu.ids gpurun_out/diag_old.txt | tail -4
fi
for v in ${AB_VARIANTS:-lean old lean old}; do
  if [ $v = old ]; then export SMCRT_LEAN=0; else unset SMCRT_LEAN; fi
  timeout -k 10 200 python3 bench.py --workload $W --no-cpu --no-ref ${BENCH_ARGS} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,2), 'M/s', round(d['ms_per_step'],2), 'ms/step', 'launch', round(d['roofline']['avg_launch_ms'],2))"
done

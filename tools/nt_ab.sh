#!/bin/bash
# Same-box A/B of bk_reduce's non-temporal record loads (base: SMCRT_RED_NT=1; nt0: plain
# loads, tools/diag_libs/libsmcrt_nt0.so): M1 throughput, then HBM bytes per kernel (PMC).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
AB_LIBS="base nt0" BENCH_ARGS="--steps 10" bash tools/ab_libs.sh || exit 1
for v in base nt0; do
  if [ $v = base ]; then unset SMCRT_LIB; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  PASSES="trace fetch write" PROF_ARGS="--no-cpu --no-ref --steps 3 --warmup 2" bash tools/profile.sh > /dev/null || exit 1
  echo "== $v"
  python3 tools/prof_summary.py gpurun_out/prof --last 3 --batch 16000000 | grep -E "lean|bk_reduce"
  rm -rf gpurun_out/prof
done

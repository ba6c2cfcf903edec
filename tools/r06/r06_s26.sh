#!/bin/bash
# Round-6 session 26: finer culling grids on M4 (SMCRT_CULL_CPT, SMCRT_CULL_MAX_CELLS), and M2's
# list reach (SMCRT_CULL_UFRAC=0 with the 4 nearest) with 6 steps per line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" "SMCRT_CULL_CPT=512" "SMCRT_CULL_CPT=1024 SMCRT_CULL_MAX_CELLS=1048576" "SMCRT_CULL_CPT=2048 SMCRT_CULL_MAX_CELLS=1048576"; do
  s=$(date +%s.%N)
  env $v timeout -k 10 300 python bench.py --workload m4 --steps 3 --warmup 1 --no-cpu --no-ref > gpurun_out/m4_cpt.json 2> gpurun_out/m4_cpt.err || { tail -5 gpurun_out/m4_cpt.err; exit 1; }
  e=$(date +%s.%N)
  python3 -c "import json,sys; d=json.load(open('gpurun_out/m4_cpt.json')); print('%-50s %7.2f M/s  run %.1f s' % (sys.argv[1] or 'base', d['value']/1e6, float(sys.argv[3])-float(sys.argv[2])))" "$v" $s $e
done
AB="base env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=4 env:SMCRT_CULL_UFRAC=0,env:SMCRT_CULL_K=6" ROUNDS=3 STEPS=6 WL=m2 bash tools/ab.sh 2>&1 | grep -v "^smoke" || exit 1

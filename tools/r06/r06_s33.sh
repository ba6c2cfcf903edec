#!/bin/bash
# Round-6 session 33: every workload line at HEAD (tools/bench_all.sh), then M5 on transport_kernel
# vs the XF lean path (r06_s32.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
STEPS=3 bash tools/bench_all.sh || exit 1
for w in m1 m0 m2 m3 m4 m5 escape; do python3 -c "import json,sys; d=json.load(open('gpurun_out/wl_%s.json'%sys.argv[1])); p=d.get('parity',{}); print('%-7s %9.2f M/s  bit-exact %s  cpu %.3f M/s' % (sys.argv[1], d['value']/1e6, p.get('counters_bit_exact_vs_cpu'), d.get('cpu_baseline',{}).get('value',0)/1e6))" $w; done
bash tools/r06/r06_s32.sh

#!/bin/bash
# Round-6 end of session 7: check at HEAD (smoke, every GPU test, bench, rocprofv3 trace + PMC into
# gpurun_out/r06_end/), then the M2 and M4 workload lines with their CPU legs (tools/bench_all.sh's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
TAG=r06_end bash tools/final_check.sh || exit 1
for w in m2 m4; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 3 --warmup 1 --cpu-seconds 8 --no-ref \
    > gpurun_out/r06_end/wl_$w.json 2> gpurun_out/r06_end/wl_$w.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), d['parity']['counters_bit_exact_vs_cpu'])" gpurun_out/r06_end/wl_$w.json $w
done

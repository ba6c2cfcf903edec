#!/bin/bash
# Round 4: every bench.py workload at HEAD (3 timed steps, 8 s CPU leg), lines to
# gpurun_out/${WL_DIR:-r04_workloads}/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/${WL_DIR:-r04_workloads}
for w in m1 m0 m2 m3 m4 m5; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 3 --warmup 1 --cpu-seconds 8 --cpu1-seconds 0 --no-ref \
    > gpurun_out/${WL_DIR:-r04_workloads}/wl_$w.json 2> gpurun_out/${WL_DIR:-r04_workloads}/wl_$w.err || { echo "$w failed"; tail -5 gpurun_out/${WL_DIR:-r04_workloads}/wl_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/${WL_DIR:-r04_workloads}/wl_$w.json'));print('$w', round(d['value']/1e6,3),'M/s', 'cpu', round(d['cpu_baseline']['value']/1e6,4), 'exact', d['parity']['counters_bit_exact_vs_cpu'])"
done
timeout -k 10 300 python -u bench.py --workload escape > gpurun_out/${WL_DIR:-r04_workloads}/wl_escape.json 2> gpurun_out/${WL_DIR:-r04_workloads}/wl_escape.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/${WL_DIR:-r04_workloads}/wl_escape.json'));print('escape', round(d['value']/1e6,3),'M/s')"

#!/bin/bash
# Round-6 GPU session: smoke, the whole GPU suite, then an M1 bench line and short M2/M5 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
NO_BENCH=1 TEST_T=900 bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py --no-ref > gpurun_out/bench_m1.json 2> gpurun_out/bench_m1.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_m1.json')); print('m1', d['value']/1e6, d['ms_per_step'], d['roofline']['avg_launch_ms'])"
for w in ${WLS:-m2 m5}; do
  timeout -k 10 240 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu --no-ref > gpurun_out/base_$w.json 2> gpurun_out/base_$w.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value']/1e6, d['ms_per_step'])" gpurun_out/base_$w.json $w
done

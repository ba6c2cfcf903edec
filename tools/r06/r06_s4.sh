#!/bin/bash
# Round-6 session 4: M5 with the COOP instantiation (far-field march for its wall-hugging
# photons) vs base: A/B (3 and 10 steps), parity via the bench's CPU leg, tail profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/tail
AB="base env:SMCRT_COOP_MIN_TOPS=1" ROUNDS=2 STEPS=3 WL=m5 bash tools/ab.sh || exit 1
AB="base env:SMCRT_COOP_MIN_TOPS=1" ROUNDS=1 STEPS=10 WL=m5 bash tools/ab.sh || exit 1
SMCRT_COOP_MIN_TOPS=1 timeout -k 10 300 python bench.py --workload m5 --steps 3 --warmup 1 --cpu-seconds 6 --cpu1-seconds 0 --no-ref > gpurun_out/m5_coop.json 2> gpurun_out/m5_coop.err || { tail gpurun_out/m5_coop.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/m5_coop.json')); print('coop m5', d['value']/1e6, d['parity'], d['roofline']['far_march_steps_per_launch'])"
SMCRT_COOP_MIN_TOPS=1 SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_diag.so SMCRT_DIAG_DONE=1 timeout -k 10 300 \
  python -u tools/tail_profile.py m5 6000000 gpurun_out/tail/m5_coop.json > gpurun_out/tail/m5_coop.txt 2>&1 || { tail -20 gpurun_out/tail/m5_coop.txt; exit 1; }
grep -v "^\[" gpurun_out/tail/m5_coop.txt | head -30

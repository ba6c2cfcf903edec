#!/bin/bash
# Round-3 session-3 GPU check: smoke, parity tests, bench, then a same-box A/B of the
# hardware-queue default (now 8) against HIP's 4 on every workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash tools/gpu_check.sh || exit 1
for wl in m1 m5 m4 m3 m0 m2; do
  st=3; [ $wl = m1 ] && st=10; [ $wl = m5 ] && st=6
  WL=$wl STEPS=$st ENVS="GPU_MAX_HW_QUEUES=4 SMCRT_SLOTS=2" bash tools/exp_env.sh | sed "s/^/$wl /" || exit 1
done

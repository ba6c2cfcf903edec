#!/bin/bash
# Same-box A/B of the number of HIP hardware queues per process (GPU_MAX_HW_QUEUES; HIP's
# default is 4, so the scene's four launch streams, its own stream, the fold stream and
# torch's stream share them and overlapped launches on one queue serialise).
# usage: WLS="m1 m5 m4" tools/hwq_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for wl in ${WLS:-m1 m5 m4}; do
  st=3; [ $wl = m1 ] && st=10
  WL=$wl STEPS=$st ENVS="${HWQ_ENVS:-GPU_MAX_HW_QUEUES=8}" bash tools/exp_env.sh || exit 1
done

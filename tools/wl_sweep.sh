#!/bin/bash
# Batch sweep of tail-bound workloads (same box): WLS="m4:8000000,16000000 m5:6000000,12000000"
# ENVS (exp_env.sh syntax) adds environment variants to each point.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
WLS=${WLS:-m4:8000000,16000000,32000000 m5:6000000,12000000,24000000}
for spec in $WLS; do
  w=${spec%%:*}
  for b in $(echo ${spec#*:} | tr ',' ' '); do
    WL=$w BATCH=$b STEPS=${STEPS:-4} bash tools/exp_env.sh | sed "s/^/$w batch $b: /" || exit 1
  done
done

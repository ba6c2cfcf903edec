#!/bin/bash
# PC sampling (host-trap) of one short bench run; output under gpurun_out/pcs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pcs
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
  --pc-sampling-interval ${PCS_INTERVAL:-50} -d gpurun_out/pcs -o pcs --output-format csv -- \
  python3 bench.py --no-cpu --steps 1 --warmup 1 --batch ${PCS_BATCH:-4000000} > gpurun_out/pcs/run.log 2>&1
rc=$?; echo "pcs rc=$rc"; find gpurun_out/pcs -type f | head; exit $rc

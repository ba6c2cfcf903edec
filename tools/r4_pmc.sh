#!/bin/bash
# Round 4: the lean kernel's stall counters (issue, instruction fetch, LDS) on M1, plus the
# counter list of this device. Output gpurun_out/r04_pmc/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_pmc
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r04_pmc/avail.txt 2>&1; echo "list rc=$?"
PASSES="${PASSES:-stall1 stall2}" PROF_ARGS="--no-cpu --no-ref --steps 2 --warmup 1" bash tools/profile.sh
rc=$?
for f in $(find gpurun_out/prof -name "*counter_collection.csv"); do cp $f gpurun_out/r04_pmc/; done
cp gpurun_out/prof/*.log gpurun_out/r04_pmc/ 2>/dev/null
exit $rc

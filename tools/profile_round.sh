#!/bin/bash
# Profile the default bench (M1) with rocprofv3: kernel trace + stats and PMC passes, then
# summarise into profiles/<TAG>/ and profiles/transport_traffic.json (read by bench.py).
# usage (on the GPU box): TAG=r02_v1 bash tools/profile_round.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
PASSES="trace sq fetch write valu" PROF_ARGS="${PROF_ARGS:---no-cpu --no-ref --steps 3 --warmup 2}" bash tools/profile.sh || exit $?
mkdir -p gpurun_out/$TAG
python3 tools/prof_summary.py gpurun_out/prof --last 3 --batch ${BATCH:-16000000} --grid ${GRID:-128} \
  --workload ${WORKLOAD:-m1} --source profiles/$TAG --json gpurun_out/$TAG/summary.json --traffic gpurun_out/$TAG/transport_traffic.json \
  > gpurun_out/$TAG/summary.txt
cat gpurun_out/$TAG/summary.txt
for p in trace pmc_sq pmc_fetch pmc_write pmc_valu; do
  f=$(find gpurun_out/prof/$p -name "*kernel_stats.csv" -o -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && cp "$f" gpurun_out/$TAG/$p.csv
done
f=$(find gpurun_out/prof/trace -name "*kernel_trace.csv" | head -1); [ -n "$f" ] && cp "$f" gpurun_out/$TAG/kernel_trace.csv
rm -rf gpurun_out/prof

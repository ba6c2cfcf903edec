#!/bin/bash
# Same-box A/B of the fold stream's priority (SMCRT_FOLD_PRIO, default high) on M1, then a
# kernel trace of the default so the fold kernels' own durations can be read.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  WL=m1 STEPS=${STEPS:-10} ENVS="SMCRT_FOLD_PRIO=0" bash tools/exp_env.sh || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prio_trace -o trace --output-format csv -- \
  python3 bench.py --no-cpu --no-ref --steps 5 --warmup 2 > gpurun_out/prio_trace.log 2>&1 || exit 1
f=$(find gpurun_out/prio_trace -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"].split("(")[0][:40]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for k, v in d.items():
    print("%-40s n=%3d avg %.3f ms max %.3f ms" % (k, len(v), sum(v) / len(v), max(v)))
EOF

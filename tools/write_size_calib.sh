#!/bin/bash
# WRITE_SIZE calibration for 8-B record stores (tools/microbench/write_size_bench.hip).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=gpurun_out/write_calib; mkdir -p $out
timeout -k 10 120 ./tools/microbench/write_size_bench > $out/plain.txt 2>&1 || exit 1
cat $out/plain.txt
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/raw -o wc --output-format csv -- ./tools/microbench/write_size_bench > $out/prof.log 2>&1 || exit 1
f=$(find $out/raw -name "*counter_collection.csv" | head -1); cp "$f" $out/counters.csv; rm -rf $out/raw
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/write_calib/counters.csv")))
for r in rows:
    print(r["Kernel_Name"][:40], r["Counter_Name"], round(float(r["Counter_Value"]) * 1024 / 1e9, 3), "GB")
PY

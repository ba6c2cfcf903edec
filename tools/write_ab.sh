#!/bin/bash
# M1 WRITE_SIZE per kernel (rocprofv3 --pmc WRITE_SIZE) for the working tree and diag_libs variants.
# usage: VARIANTS="ntlast ntall" bash tools/write_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/write_ab
for v in new $VARIANTS; do
  if [ $v = new ]; then unset SMCRT_LIB; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/write_ab/raw_$v -o w --output-format csv -- \
    python3 bench.py --no-cpu --no-ref --steps 3 --warmup 1 > gpurun_out/write_ab/b_$v.json 2> gpurun_out/write_ab/b_$v.err || { echo "$v failed"; exit 1; }
  f=$(find gpurun_out/write_ab/raw_$v -name "*counter_collection.csv" | head -1); cp "$f" gpurun_out/write_ab/wc_$v.csv; rm -rf gpurun_out/write_ab/raw_$v
  python3 - $v <<'PY'
import csv, sys, collections
v = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/write_ab/wc_{v}.csv")))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"].split("(")[0][:30]].append(float(r["Counter_Value"]) * 1024)
for k, xs in agg.items():
    if max(xs) > 1e9:
        big = [x for x in xs if x > 1e9]
        print(f"{v:8s} {k:30s} n={len(big)} mean {sum(big)/len(big)/1e9:.2f} GB per dispatch")
PY
done
for v in new $VARIANTS; do
  if [ $v = new ]; then unset SMCRT_LIB; else export SMCRT_LIB=$PWD/tools/diag_libs/libsmcrt_$v.so; fi
  timeout -k 10 200 python3 bench.py --no-cpu --no-ref --steps 10 --warmup 2 > gpurun_out/write_ab/t_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/write_ab/t_$v.json'));print('$v', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],1), 'ms/step')"
done

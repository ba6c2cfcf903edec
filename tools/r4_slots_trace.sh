#!/bin/bash
# Kernel traces of the M1 bench with two and three record slots (the fold's place in the timeline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
for sl in 2 3; do
  out=gpurun_out/slots$sl; mkdir -p $out
  SMCRT_SLOTS=$sl timeout -k 10 300 rocprofv3 --kernel-trace -d $out/raw -o tr --output-format csv -- \
    python3 bench.py --no-cpu --no-ref --steps 4 --warmup 2 > $out/bench.json 2> $out/bench.err || exit 1
  f=$(find $out/raw -name "*kernel_trace.csv" | head -1); cp "$f" $out/kernel_trace.csv; rm -rf $out/raw
  python3 -c "import json;d=json.load(open('$out/bench.json'));print('slots $sl', d['value'], d['ms_per_step'])"
done

#!/bin/bash
# Build compile-time variants of the engine into tools/diag_libs/libsmcrt_NAME.so (CPU, no GPU
# needed; every unit is compiled with the flags). usage: tools/variants.sh NAME "-DFOO=1" [NAME2 "FLAGS2" ...]
cd "$(dirname "$0")/.." || exit 1
python3 -m rsmcrt_amd.build --variant "$@" > /tmp/smcrt_variants.log 2>&1 || { tail -20 /tmp/smcrt_variants.log; exit 1; }
ls -la tools/diag_libs/

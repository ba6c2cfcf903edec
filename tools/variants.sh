#!/bin/bash
# Build compile-time variants of the engine into tools/diag_libs/ (CPU, no GPU needed).
# usage: tools/variants.sh NAME "-DFOO=1 -DBAR=2" [NAME2 "FLAGS2" ...]
cd "$(dirname "$0")/.." || exit 1
python3 -m rsmcrt_amd.build --variant "$@" && ls -la tools/diag_libs/

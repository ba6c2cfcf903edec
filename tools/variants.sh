#!/bin/bash
# Build compile-time variants of the engine into tools/diag_libs/ (CPU, no GPU needed).
# usage: tools/variants.sh NAME "-DFOO=1 -DBAR=2" [NAME2 "FLAGS2" ...]
cd "$(dirname "$0")/.." || exit 1
mkdir -p tools/diag_libs
SRCS=$(python3 -c "import sys; sys.path.insert(0, '.'); from rsmcrt_amd import build as B; print(' '.join(B.SOURCES))")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 $flags \
    -o tools/diag_libs/libsmcrt_$name.so $SRCS -lz &
done
wait
ls -la tools/diag_libs/

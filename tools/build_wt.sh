#!/bin/bash
# Build the engine library of the WORKING TREE into tools/diag_libs/libsmcrt_<name>.so with
# extra hipcc flags, for same-box A/B timing (tools/ab_libs.sh).
# usage: tools/build_wt.sh NAME [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/diag_libs
srcs=$(python3 -c "import sys; sys.path.insert(0, '.'); from rsmcrt_amd import build as B; print(' '.join(B.SOURCES))")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 "$@" \
  -o tools/diag_libs/libsmcrt_$name.so $srcs -lz -ldl

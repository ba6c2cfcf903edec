#!/bin/bash
# Build the engine library of a git revision into tools/diag_libs/libsmcrt_<name>.so, for
# same-box A/B timing against the working tree (tools/sweep.sh).  usage: build_ref_variant.sh REV NAME
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; tmp=$(mktemp -d)
mkdir -p $tmp/rsmcrt_amd/csrc $tmp/include tools/diag_libs
for f in rsmcrt_amd/csrc/smcrt.hip rsmcrt_amd/csrc/transport.h rsmcrt_amd/csrc/detmath.h rsmcrt_amd/csrc/geometry.h \
         rsmcrt_amd/csrc/deposit.h include/smcrt.h; do
  git show $rev:$f > $tmp/$f
done
srcs=$tmp/rsmcrt_amd/csrc/smcrt.hip
for f in rsmcrt_amd/csrc/hosterr.h rsmcrt_amd/csrc/writers.cpp; do  # newer revisions only
  git show $rev:$f > $tmp/$f 2>/dev/null || rm -f $tmp/$f
done
[ -f $tmp/rsmcrt_amd/csrc/writers.cpp ] && srcs="$srcs $tmp/rsmcrt_amd/csrc/writers.cpp"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -o tools/diag_libs/libsmcrt_$name.so $srcs
rm -rf $tmp

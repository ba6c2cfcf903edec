#!/bin/bash
# Build the engine library of a git revision (a temporary worktree) into
# tools/diag_libs/libsmcrt_<name>.so, for same-box A/B timing (tools/sweep.sh).
# usage: tools/build_rev.sh REV NAME [extra hipcc flags...]
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
git worktree add -q --detach $tmp $rev
mkdir -p tools/diag_libs
srcs=$(cd $tmp && python3 -c "import sys; sys.path.insert(0, '.'); from rsmcrt_amd import build as B; print(' '.join(B.SOURCES))")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off -fno-fast-math --offload-arch=gfx950 "$@" \
  -o tools/diag_libs/libsmcrt_$name.so $srcs -lz -ldl
git worktree remove --force $tmp

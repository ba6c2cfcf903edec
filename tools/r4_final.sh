#!/bin/bash
# Round 4 check at HEAD: smoke, every GPU test, bench (M1), then the rocprofv3 profile of the
# bench (kernel trace + PMC passes) into gpurun_out/r04_final/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TEST_T=900 bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/r04_final
cp gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench.json gpurun_out/bench.err gpurun_out/r04_final/
TAG=r04_final bash tools/profile_round.sh > gpurun_out/r04_final/profile.log 2>&1
rc=$?; tail -8 gpurun_out/r04_final/profile.log; exit $rc

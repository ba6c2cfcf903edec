#!/bin/bash
# Check at HEAD: smoke, every GPU test, bench (M1), then the rocprofv3 profile of the bench
# (kernel trace + PMC passes) into gpurun_out/$TAG/. usage: TAG=r04_s3 bash tools/final_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:?set TAG}
TEST_T=900 bash tools/gpu_check.sh || exit 1
mkdir -p gpurun_out/$TAG
cp gpurun_out/smoke.log gpurun_out/pytest_gpu.log gpurun_out/bench.json gpurun_out/bench.err gpurun_out/$TAG/
[ -n "$NO_PROFILE" ] && exit 0
TAG=$TAG bash tools/profile_round.sh > gpurun_out/$TAG/profile.log 2>&1
rc=$?; tail -8 gpurun_out/$TAG/profile.log; exit $rc

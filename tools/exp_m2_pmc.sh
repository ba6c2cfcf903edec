#!/bin/bash
# M2 (40-sphere scene) tail diagnostics: one small launch under two PMC passes, so that
# instructions and cycles per wave-trip can be read off (wave_iterations_per_launch in the
# bench line). Output under gpurun_out/m2pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/m2pmc; mkdir -p $O
B=${M2_BATCH:-20000}
ARGS="--workload m2 --batch $B --steps 1 --warmup 1 --no-cpu --no-ref --overlap 0"
timeout -k 10 200 python3 bench.py $ARGS > $O/bench.json 2> $O/bench.err || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY \
  -d $O/p1 -o p1 --output-format csv -- python3 bench.py $ARGS > $O/p1.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_FLAT \
  -d $O/p2 -o p2 --output-format csv -- python3 bench.py $ARGS > $O/p2.log 2>&1 || exit $?
find $O -name "*counter_collection.csv" -exec cp {} $O/ \;
echo done

#!/bin/bash
# rocprofv3 passes over a short bench run: kernel trace + stats, then PMC counters in
# separate passes (never combined with runtime/sys tracing). Output under gpurun_out/prof.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${PROF_ARGS:-"--no-cpu --steps 3 --warmup 2"}
fatal() { [ "$1" -ge 124 ] || [ "$1" -eq 134 ] || [ "$1" -eq 139 ]; }
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
    > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; if fatal $rc; then exit $rc; fi
}
PASSES=${PASSES:-"trace sq fetch write tcc"}
for p in $PASSES; do
  case $p in
    trace) run trace --kernel-trace --stats ;;
    sq) run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE ;;
    fetch) run pmc_fetch --pmc FETCH_SIZE ;;
    write) run pmc_write --pmc WRITE_SIZE ;;
    tcc) run pmc_tcc --pmc TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum ;;
    stall1) run pmc_stall1 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM ;;
    stall2) run pmc_stall2 --pmc SQ_IFETCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_SENDMSG ;;
    valu) run pmc_valu --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_SMEM ;;
  esac
done
find $OUT -name "*.csv" | head -50

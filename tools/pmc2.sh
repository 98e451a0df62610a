# Memory-pipeline / issue PMC passes (TA, TCP, SQ), each in its own rocprofv3 run.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc2
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
pass() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -3 $OUT/$name.log; fi
  if [ $rc -ge 128 ]; then exit $rc; fi
  return 0
}
pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
pass tcp2 TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum
pass sqa SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM SQ_IFETCH SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES
pass sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_IFETCH_LEVEL SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE
pass sqc SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
echo done

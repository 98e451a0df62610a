# Issue/stall PMC passes (SQ) for the current build.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc3
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline"
pass() {
  name=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$OUT/$name -o run --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ge 128 ]; then exit $rc; fi
  return 0
}
pass sqa SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM
pass sqb SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE
pass sqc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT64 SQ_INSTS_SMEM
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo done

# rocprofv3 PMC passes (counters only, each in its own run) over a short bench run.
# Outputs gpurun_out/pmc/<pass>/run_counter_collection.csv.  Stops on a fault/abort/timeout.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline ${PMC_BENCH_ARGS:-}"
pass() {
  name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$name -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$name.log; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE
pass tcc TCC_HIT_sum TCC_MISS_sum
echo done

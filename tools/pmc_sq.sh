# Two rocprofv3 SQ counter passes over a short C2 bench run (each pass its own run); summary per kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
rm -rf gpurun_out/pmc/*
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --no-cpu-baseline ${PMC_BENCH_ARGS:-}"
pass() {
  name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/gpurun_out/pmc/$name -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc/$name.log 2>&1
  rc=$?
  echo "pass $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/$name.log; exit $rc; fi
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
python3 tools/pmc_summary.py gpurun_out/pmc --json gpurun_out/pmc/summary.json > /dev/null
python3 tools/pmc_brief.py gpurun_out/pmc/summary.json

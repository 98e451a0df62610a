# one SQ counter pass over a short bench (args: bench args)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/pmcq; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d $GRAFT_REPO_ROOT/gpurun_out/pmcq/sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmcq/sq.log 2>&1 || exit 4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pmcq/kt -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > gpurun_out/pmcq/kt.log 2>&1 || exit 4
echo ok

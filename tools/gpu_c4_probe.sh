# C4 closest-hit investigation: traversal work per ray (profiling build), per-launch kernel
# trace, and PMC passes (fetch / write / L2 hit-miss) of the C4 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4probe
export TMPDIR=/tmp
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 300 python tools/trav_stats.py c4 --json gpurun_out/c4probe/trav_c4.json > gpurun_out/c4probe/trav.log 2>&1 || { tail -5 gpurun_out/c4probe/trav.log; exit 3; }
cat gpurun_out/c4probe/trav.log | tail -3
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c4probe/kt -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c4probe/kt.log 2>&1 || { tail -5 gpurun_out/c4probe/kt.log; exit 4; }
tail -1 gpurun_out/c4probe/kt.log | cut -c1-400
python3 tools/ktrace.py gpurun_out/c4probe/kt k_closest k_shadow k_shade
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/gpurun_out/c4probe/pmc_$name -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/c4probe/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -3 gpurun_out/c4probe/pmc_$name.log; exit 5; }
  echo "pmc $name ok"
done

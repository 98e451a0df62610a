# C4 closest-hit: wide vs quantised nodes, kernel trace + TA/TCP counters of each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4fmt
export TMPDIR=/tmp
export PBRT_C4_DIR=/tmp/c4scene
B="python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --spp 32"
for fmt in wide compressed; do
  export PBRT_AMD_BVH=$fmt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c4fmt/kt_$fmt -o run --output-format csv -- $B > gpurun_out/c4fmt/kt_$fmt.log 2>&1 || { tail -5 gpurun_out/c4fmt/kt_$fmt.log; exit 4; }
  echo "== $fmt"; python3 tools/ktrace.py gpurun_out/c4fmt/kt_$fmt k_closest k_shadow
  for pass in "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum" "FETCH_SIZE"; do
    name=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 200 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/gpurun_out/c4fmt/$fmt/pmc_$name -o run --output-format csv -- $B > gpurun_out/c4fmt/pmc_${fmt}_$name.log 2>&1 || { echo "pmc $name failed"; tail -3 gpurun_out/c4fmt/pmc_${fmt}_$name.log; exit 5; }
  done
  python3 tools/pmc_summary.py gpurun_out/c4fmt/$fmt | grep -A14 k_closest
done

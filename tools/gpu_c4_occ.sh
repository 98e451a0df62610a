# C4 closest-hit / shadow per-launch times: traversal occupancy (4/5/6 blocks per CU) x node format
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c4occ
export TMPDIR=/tmp
export PBRT_C4_DIR=/tmp/c4scene
B="python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline --spp 32"
for w in 4 5 6; do
  for fmt in wide compressed; do
    if [ $w -eq 4 ]; then export PBRT_AMD_LIB=$GRAFT_REPO_ROOT/pbrt-v4_amd/lib/libpbrt_amd.so; else export PBRT_AMD_LIB=$GRAFT_REPO_ROOT/pbrt-v4_amd/lib/libpbrt_amd_w$w.so; fi
    export PBRT_AMD_BVH=$fmt
    d=gpurun_out/c4occ/kt_${w}_$fmt
    timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$d -o run --output-format csv -- $B > $d.log 2>&1 || { tail -5 $d.log; exit 4; }
    echo "== w$w $fmt $(tail -1 $d.log | cut -c70-110)"; python3 tools/ktrace.py $d k_closest k_shadow
  done
done

set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in libpbrt_amd libpbrt_amd_fasttrig; do
  PBRT_AMD_LIB=$GRAFT_REPO_ROOT/pbrt-v4_amd/lib/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/exp_$lib -o run --output-format csv -- python3 bench.py --workload c5 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/exp_$lib.log 2>&1 || exit 4
  echo $lib; grep -h "k_v" gpurun_out/exp_$lib/*kernel_stats.csv | cut -d, -f1-4 | sed 's/(pbrt_amd::DeviceScene, pbrt_amd::PathState, pbrt_amd::VolState, int)//'
done

# Run bench.py once per library variant (lib/exp_*.so) on the GPU box, then a rocprofv3 kernel
# summary of each: tools/kstats.py prints per-kernel mean launch time.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_*.so; do
  [ -f "$lib" ] || continue
  n=$(basename $lib .so)
  PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/$n.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/var/$n.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/var/$n.log').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"
  if [ -n "$PROF" ]; then
    PBRT_AMD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/var/prof_$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/prof_$n.log 2>&1 || { echo "prof $n failed"; exit 3; }
    python3 tools/kstats.py gpurun_out/var/prof_$n
  fi
done

# C2 4-wave shade A/B (lib/exp_w4.so: PBRT_SHADE_WAVES=4) and the C3 k_closest PMC record.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6f
mkdir -p $O
export TMPDIR=/tmp
for lib in libpbrt_amd exp_w4; do
  PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/$lib.so timeout -k 10 120 python -u tools/film_hash.py > $O/hash_$lib.log 2>&1 || { echo "hash $lib failed"; tail -3 $O/hash_$lib.log; exit 3; }
  echo "$lib $(tail -1 $O/hash_$lib.log)"
  PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/$lib.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_$lib.log 2>&1 || { echo "bench $lib failed"; tail -3 $O/c2_$lib.log; exit 3; }
  tail -1 $O/c2_$lib.log | cut -c1-200
done
PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/exp_w4.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_w4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_w4.log 2>&1 || { echo "rocprof failed"; tail -3 $O/prof_w4.log; exit 4; }
HEAD_SHA=${HEAD_SHA:-unknown} bash tools/gpu_r6_pmc.sh r6f "c3"

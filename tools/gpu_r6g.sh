# Round-6 check after HitTextures was force-inlined: textured GPU tests first (the k_texture
# hang), the whole -m gpu suite, the C2 4-wave shade A/B (lib/exp_w4.so) with a kernel trace of
# the variant, then the C4 / C3 k_closest PMC records.  Stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_textures.py tests/test_vol_textures.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tex.log 2>&1 || { echo "textured tests failed"; tail -15 $O/tex.log; exit 3; }
tail -1 $O/tex.log
bash tools/gpu_r6.sh r6g tests "" "" || exit $?
for lib in libpbrt_amd exp_w4; do
  PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/$lib.so timeout -k 10 120 python -u tools/film_hash.py > $O/hash_$lib.log 2>&1 || { echo "hash $lib failed"; tail -3 $O/hash_$lib.log; exit 3; }
  echo "$lib $(tail -1 $O/hash_$lib.log)"
  PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/$lib.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2_$lib.log 2>&1 || { echo "bench $lib failed"; tail -3 $O/c2_$lib.log; exit 3; }
  tail -1 $O/c2_$lib.log | cut -c1-200
done
PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/exp_w4.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_w4 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_w4.log 2>&1 || { echo "rocprof failed"; tail -3 $O/prof_w4.log; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_main -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_main.log 2>&1 || { echo "rocprof failed"; tail -3 $O/prof_main.log; exit 4; }
HEAD_SHA=${HEAD_SHA:-unknown} bash tools/gpu_r6_pmc.sh r6g "c4 c3"

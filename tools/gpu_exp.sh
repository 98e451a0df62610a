# Build-variant experiment round trip: the device self-checks (exact math forms), film hashes of
# every variant (bit-identical to the default build?) and a bench line per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_rn_math.py > gpurun_out/rn.log 2>&1; rc=$?
tail -3 gpurun_out/rn.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_*.so; do
  [ -f "$lib" ] || continue
  for sc in ${FILM_SCENES:-cornell c3}; do
    PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/film_hash.py $sc > gpurun_out/var/hash.log 2>&1 || { echo "$lib hash failed"; tail -3 gpurun_out/var/hash.log; exit 3; }
    echo "$(basename $lib) $(tail -1 gpurun_out/var/hash.log)"
  done
done
bash tools/bench_variants.sh

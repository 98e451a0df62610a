# Round-6: textured subsurface spectra -- the subsurface and hair GPU parity forms first, then the
# whole -m gpu suite and the C2 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 600 python -u -m pytest tests/test_subsurface.py tests/test_hair.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $O/sss.log 2>&1; rc=$?
grep -E "subsurface \(|hair \(|passed|failed" $O/sss.log | tail -16
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r6.sh r6t tests "c2" "" || exit $?

# Round-6: textured hair floats -- the hair GPU parity forms first, then the whole -m gpu suite,
# and the C2 bench line (no change expected: lean kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 600 python -u -m pytest tests/test_hair.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $O/hair.log 2>&1; rc=$?
grep -E "hair \(|passed|failed" $O/hair.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r6.sh r6s tests "c2" "" || exit $?

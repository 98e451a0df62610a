# Round-6: the new GPU tests (bump maps on the volumetric materials, textured hair), then the suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bump_volumetric.py tests/test_hair.py tests/test_textures.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -s > $O/new.log 2>&1; rc=$?
grep -E "parity|hair \(|passed|failed" $O/new.log | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r6.sh r6h tests "" ""

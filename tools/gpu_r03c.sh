# texture GPU tests first, then every GPU test, then the C2 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_textures.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c/tex.log 2>&1; rc=$?
echo "texture gpu rc=$rc"; grep -E "PASS|FAIL|parity|Error" gpurun_out/r03c/tex.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03c/all.log 2>&1; rc2=$?
echo "all gpu rc=$rc2"; tail -4 gpurun_out/r03c/all.log
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03c/c2.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r03c/c2.log; exit 3; }
tail -1 gpurun_out/r03c/c2.log | cut -c1-300

# mix + texture GPU tests, C4 textured bench line (k_texture LDS staging), rocprofv3 kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_mix.py tests/test_textures.py -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "parity|passed|failed|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 500 python bench.py --workload c4 --steps 2 --warmup 1 > $O/c4tex.log 2>&1 || { echo "c4 bench failed"; tail -5 $O/c4tex.log; exit 3; }
tail -1 $O/c4tex.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 4; }
echo rocprof ok

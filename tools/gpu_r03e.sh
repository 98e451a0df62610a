# texture + C4 GPU tests, C4 textured bench line, rocprofv3 kernel summary of it
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_textures.py tests/test_gpu_parity.py -k "textur or c4" -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03e/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "parity|passed|failed|Error" gpurun_out/r03e/tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 500 python bench.py --workload c4 --steps 2 --warmup 1 ${C4ARGS} > gpurun_out/r03e/c4tex.log 2>&1 || { echo "c4 bench failed"; tail -5 gpurun_out/r03e/c4tex.log; exit 3; }
tail -1 gpurun_out/r03e/c4tex.log | cut -c1-200
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03e/prof -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03e/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r03e/prof.log; exit 4; }
echo rocprof ok

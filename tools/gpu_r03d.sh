# C4 textured: parity tests, bench lines (textured and untextured), rocprofv3 kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k c4 -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03d/c4tests.log 2>&1; rc=$?
echo "c4 tests rc=$rc"; grep -E "PASS|FAIL|parity|Error" gpurun_out/r03d/c4tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 500 python bench.py --workload c4 --steps 2 --warmup 1 > gpurun_out/r03d/c4tex.log 2>&1 || { echo "c4 bench failed"; tail -5 gpurun_out/r03d/c4tex.log; exit 3; }
tail -1 gpurun_out/r03d/c4tex.log | cut -c1-400
export PBRT_C4_DIR=/tmp/c4scene_u
timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 --untextured --no-cpu-baseline > gpurun_out/r03d/c4untex.log 2>&1 || { echo "c4 untex failed"; tail -5 gpurun_out/r03d/c4untex.log; exit 3; }
tail -1 gpurun_out/r03d/c4untex.log | cut -c1-300
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03d/prof -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03d/prof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/r03d/prof.log; exit 4; }
echo rocprof ok

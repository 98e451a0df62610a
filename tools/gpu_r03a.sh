# GPU tests (incl. the full-size C4 intersections / stripe), then C2 and C4 bench lines and a C4
# per-launch kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03a/pytest_gpu.log 2>&1; rc=$?
echo "gpu pytest rc=$rc"; grep -E "C4 full|passed|failed|Error" gpurun_out/r03a/pytest_gpu.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r03a/bench_c2.log 2>&1 || exit 3
tail -1 gpurun_out/r03a/bench_c2.log | cut -c1-250
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03a/kt_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03a/kt_c4.log 2>&1 || { tail -5 gpurun_out/r03a/kt_c4.log; exit 4; }
tail -1 gpurun_out/r03a/kt_c4.log | cut -c1-250
python3 tools/ktrace.py gpurun_out/r03a/kt_c4 k_closest k_shadow k_shade

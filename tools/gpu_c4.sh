# GPU tests, the C4 bench line (with CPU baseline) and a rocprofv3 kernel summary of C4.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "parity|passed|failed|Error" gpurun_out/pytest_gpu.log | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_c4.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c4.log; exit 3; }
tail -1 gpurun_out/bench_c4.log | cut -c1-1600
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c4.log; exit 4; }
echo "rocprof ok"
find gpurun_out/prof_c4 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -14

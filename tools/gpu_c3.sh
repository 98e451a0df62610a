# C3 bench line (with CPU baseline) + rocprofv3 kernel statistics of a short C3 run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload c3 ${C3_ARGS} > gpurun_out/bench_c3.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c3.log; exit 3; }
tail -1 gpurun_out/bench_c3.log | cut -c1-1500
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c3.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c3.log; exit 4; }
echo "rocprof ok"
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -20

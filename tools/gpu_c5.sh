# C5 (media) bench line + rocprofv3 kernel summary.  $1 = spp (default 64 for a quick look)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SPP=${1:-64}
timeout -k 10 600 python -u bench.py --workload c5 --spp $SPP --steps ${2:-2} --warmup 1 > gpurun_out/bench_c5.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c5.log; exit 3; }
tail -1 gpurun_out/bench_c5.log | cut -c1-1500
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --workload c5 --spp 16 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c5.log; exit 4; }
echo "rocprof ok"
find gpurun_out/prof_c5 -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -14

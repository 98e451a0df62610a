# smoke(), the default C2 bench line, and a rocprofv3 kernel-trace summary of the same bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.log 2>&1 || { tail -5 gpurun_out/bench_c2.log; exit 3; }
tail -1 gpurun_out/bench_c2.log | cut -c1-700
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1 || { tail -5 gpurun_out/prof_c2.log; exit 3; }
find gpurun_out/prof_c2 -name "*kernel_stats.csv" | head -3
tail -1 gpurun_out/prof_c2.log | cut -c1-400

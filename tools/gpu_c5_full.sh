# C5 at its full configuration (1280x720, 1024 spp): bench line + rocprofv3 kernel summary
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_media.py -q --timeout 300 --timeout-method thread > gpurun_out/pytest_media.log 2>&1 || { tail -5 gpurun_out/pytest_media.log; exit 2; }
tail -1 gpurun_out/pytest_media.log
timeout -k 10 900 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/bench_c5_full.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_c5_full.log; exit 3; }
tail -1 gpurun_out/bench_c5_full.log
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c5_full -o run --output-format csv -- python3 bench.py --workload c5 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5_full.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_c5_full.log; exit 4; }
tail -1 gpurun_out/prof_c5_full.log | cut -c1-300
cat gpurun_out/prof_c5_full/run_kernel_stats.csv | cut -d, -f1-5 | head -12

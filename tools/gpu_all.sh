# every GPU test, then the C2 bench line, the C5 bench line and the C3 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "gpu pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit 3
tail -1 gpurun_out/bench_c2.log | cut -c1-200
timeout -k 10 600 python bench.py --workload c5 --spp 64 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1 || exit 3
tail -1 gpurun_out/bench_c5.log | cut -c1-200
timeout -k 10 600 python bench.py --workload c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1 || exit 3
tail -1 gpurun_out/bench_c3.log | cut -c1-200

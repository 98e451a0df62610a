# GPU round trip for a feature change: every gpu test (with parity prints), then the C2 bench
# line.  A test assertion failure (rc 1) still lets the bench run; a fault, abort or timeout
# ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "parity|passed|failed|Error|assert" gpurun_out/pytest_gpu.log | tail -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log | cut -c1-600

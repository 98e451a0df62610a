# Round-6 GPU check: bash tools/gpu_r6.sh TAG "PYTEST-ARGS|-" "BENCH-WORKLOADS" [PROFILE-WORKLOAD]
# Runs the -m gpu tests (one process, each test under pytest-timeout), then one bench line per
# workload, then (optionally) a rocprofv3 kernel-trace summary of one workload.  Output under
# gpurun_out/TAG/.  Every GPU step has its own time limit and the script stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; TESTS=$2; BENCHES=$3; PROF=$4
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
if [ "$TESTS" != "-" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -2; grep -E "FAILED|Error" $O/tests.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for w in $BENCHES; do
  timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $O/bench_$w.log; exit 3; }
  tail -1 $O/bench_$w.log | cut -c1-220
done
if [ -n "$PROF" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --workload $PROF --steps 2 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 4; }
  echo "rocprof ok"; find $O/prof -name "*kernel_stats.csv" | head -2
fi

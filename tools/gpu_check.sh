# Generic GPU check: bash tools/gpu_check.sh TAG "PYTEST-ARGS" "BENCH-WORKLOADS" [profile]
# Runs the given -m gpu tests, then one bench line per workload (c2, c4, ...), then (with a
# 4th argument) a rocprofv3 kernel summary of the last workload.  Output: gpurun_out/TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; TESTS=$2; BENCHES=$3; PROF=$4
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "parity|passed|failed|Error|bounce" $O/tests.log | tail -25
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
last=""
for w in $BENCHES; do
  timeout -k 10 500 python bench.py --workload $w --steps 3 --warmup 1 > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $O/bench_$w.log; exit 3; }
  tail -1 $O/bench_$w.log | cut -c1-160
  last=$w
done
if [ -n "$PROF" ] && [ -n "$last" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 bench.py --workload $last --steps 1 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/prof.log; exit 4; }
  echo rocprof ok
fi

set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "passed|failed" $O/tests.log | tail -3; grep -E "FAILED|parity|libm|correctly rounded" $O/tests.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in c2 c5; do
  timeout -k 10 500 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $O/bench_$w.log; exit 3; }
  tail -1 $O/bench_$w.log | cut -c1-200
done

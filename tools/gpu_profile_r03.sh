# Round-3 profile set: selected GPU tests, then C2 and C4 bench lines with rocprofv3 kernel
# summaries and the C4 closest-hit PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "$1" > $O/pytest.log 2>&1; rc=$?
  echo "tests rc=$rc"; grep -E "FAILED|^E |passed|failed" $O/pytest.log | tail -8
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py > $O/bench_c2.log 2>&1 || exit 3
tail -1 $O/bench_c2.log > $O/r03_c2_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_c2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_c2.log 2>&1 || exit 4
export PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 > $O/bench_c4.log 2>&1 || exit 5
tail -1 $O/bench_c4.log > $O/r03_c4_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/kt_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/kt_c4.log 2>&1 || exit 6
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $pass -d $GRAFT_REPO_ROOT/$O/pmc_c4/$name -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 0 --no-cpu-baseline > $O/pmc_c4_$name.log 2>&1 || { echo "pmc $name failed"; exit 7; }
done
echo "profile set ok"
python3 -c "import json; [print(f, json.load(open('$O/'+f))['value']) for f in ('r03_c2_bench.json','r03_c4_bench.json')]"

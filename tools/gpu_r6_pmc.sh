# Round-6 k_closest traffic records: bash tools/gpu_r6_pmc.sh TAG "WORKLOADS"
# Per workload: one bench line, the film hash of a small render (c4 / c3), then FETCH_SIZE,
# WRITE_SIZE and TCC hit/miss passes (each its own rocprofv3 run, counters only) of a one-step
# bench, summarised per k_closest launch by tools/c4_pmc_json.py.  Output under gpurun_out/TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; WLS=$2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for w in $WLS; do
  timeout -k 10 600 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $O/bench_$w.log; exit 3; }
  tail -1 $O/bench_$w.log > $O/bench_$w.json
  cut -c1-300 $O/bench_$w.json
  timeout -k 10 300 python tools/film_hash.py $w > $O/hash_$w.log 2>&1 || { echo "hash $w failed"; tail -5 $O/hash_$w.log; exit 3; }
  tail -1 $O/hash_$w.log
  mkdir -p $O/pmc_$w
  for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "tcc TCC_HIT_sum TCC_MISS_sum"; do
    set -- $p
    n=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$O/pmc_$w/$n -o run --output-format csv -- python3 bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_$w/$n.log 2>&1 || { echo "pmc $w $n failed"; tail -5 $O/pmc_$w/$n.log; exit 3; }
  done
  for n in fetch write tcc; do f=$(find $O/pmc_$w/$n -name "*counter_collection.csv" | head -1); mkdir -p $O/pmcx_$w/$n; cp $f $O/pmcx_$w/$n/run_counter_collection.csv; done
  python3 tools/c4_pmc_json.py $O/pmcx_$w $O/bench_$w.json $O/closest_pmc_$w.json ${HEAD_SHA:-unknown} "$w" > /dev/null && head -14 $O/closest_pmc_$w.json
done

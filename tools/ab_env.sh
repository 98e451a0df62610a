#!/bin/bash
# A/B of one environment switch of the same library (tools only): film hash per value
# (bit-identity), then one bench line per value.
# Usage: VAR=PBRT_AMD_XCD_GROUPS VALUES="1 0" HASH_ARGS="cornell 320 180 16" BENCH_ARGS="--workload c4" bash tools/ab_env.sh TAG
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
tag=${1:-ab}
for v in $VALUES; do
  env "$VAR=$v" timeout -k 10 150 python -u tools/film_hash.py ${HASH_ARGS:-} > gpurun_out/var/${tag}_hash_$v.txt 2>&1 || { echo "hash $v failed"; tail -3 gpurun_out/var/${tag}_hash_$v.txt; exit 3; }
  echo "$VAR=$v: $(tail -1 gpurun_out/var/${tag}_hash_$v.txt)"
done
for v in $VALUES; do
  env "$VAR=$v" timeout -k 10 400 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/${tag}_bench_$v.json 2> gpurun_out/var/${tag}_bench_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/var/${tag}_bench_$v.err; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/var/${tag}_bench_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', d['value'], d['ms_per_step'], r.get('mean_launch_us'))"
done

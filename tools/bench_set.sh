#!/bin/bash
# Benches of the secondary workloads (tools only): bash tools/bench_set.sh TAG "c2 c3 c4 c5".
# Outputs gpurun_out/bench_<TAG>_<workload>.json; stops at the first failing run.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=$1
for w in ${2:-c2 c3 c4 c5}; do
  steps=5; [ $w = c4 ] && steps=3; [ $w = c5 ] && steps=3
  timeout -k 10 500 python3 -u bench.py --workload $w --steps $steps --warmup 1 --no-cpu-baseline \
    > gpurun_out/bench_${tag}_$w.json 2> gpurun_out/bench_${tag}_$w.err || { tail -5 gpurun_out/bench_${tag}_$w.err; exit 3; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_${tag}_$w.json')); print('$w', d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"
done

# Bench lines of the secondary workloads (C3, C4, C5) plus kernel summaries.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wl
export TMPDIR=/tmp
for wl in ${WORKLOADS:-c3 c4 c5}; do
  timeout -k 10 400 python bench.py --workload $wl ${CPU_BASELINE:---no-cpu-baseline} ${BENCH_ARGS:-} > gpurun_out/wl/$wl.log 2>&1 || { echo "$wl failed"; tail -5 gpurun_out/wl/$wl.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/wl/$wl.log').read().strip().splitlines()[-1]); print('$wl', d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'], d['roofline']['frac'])"
  if [ -n "$PROF" ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/wl/prof_$wl -o run --output-format csv -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/wl/prof_$wl.log 2>&1 || { echo "prof $wl failed"; exit 3; }
    python3 tools/kstats.py gpurun_out/wl/prof_$wl
  fi
done

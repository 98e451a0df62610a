# Round-6 closing records: smoke(), then rocprofv3 kernel-trace summaries of C3, C4 and C5 at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6v
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for w in c3 c4 c5; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$w -o run --output-format csv -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$w.log 2>&1 || { echo "rocprof $w failed"; tail -5 $O/prof_$w.log; exit 4; }
  echo "rocprof $w ok"
done

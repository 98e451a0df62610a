# Round-6: traversal occupancy A/B (k_closest / k_shadow compiled for 4 = default, 5 and 6 waves
# per SIMD: lib/libpbrt_amd_w5.so, _w6.so), C2 / C3 bench lines plus per-kernel rocprofv3
# summaries of C2; then the traversal work per ray at HEAD (profiling build).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for v in w4 w5 w6; do
  lib=$PWD/pbrt-v4_amd/lib/libpbrt_amd.so; [ $v != w4 ] && lib=$PWD/pbrt-v4_amd/lib/libpbrt_amd_$v.so
  for w in c2 c3; do
    PBRT_AMD_LIB=$lib timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_$v.log 2>&1 || { echo "bench $w $v failed"; tail -3 $O/${w}_$v.log; exit 3; }
    tail -1 $O/${w}_$v.log > $O/${w}_$v.json
    python3 -c "import json; d=json.load(open('$O/${w}_$v.json')); r=d['roofline']; print('$w $v', d['value'], r.get('mean_launch_us'))"
  done
  PBRT_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run --output-format csv -- python3 bench.py --workload c2 --steps 2 --warmup 1 --no-cpu-baseline > $O/prof_$v.log 2>&1 || { echo "rocprof $v failed"; tail -5 $O/prof_$v.log; exit 4; }
  python3 - $O/prof_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "k_closest" in n or "k_shadow" in n or "k_shade_diffuse" in n:
        print("  ", n[:40], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
timeout -k 10 300 python tools/trav_stats.py c2 --json $O/r06_c2_trav_stats.json > $O/trav.log 2>&1 || { tail -5 $O/trav.log; exit 5; }
tail -3 $O/trav.log

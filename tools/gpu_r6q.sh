# Round-6: the -m gpu suite at HEAD (k_shadow at 5 waves in the all-LDS mode, plymesh
# displacement), C2 bench + rocprofv3 summary with the default library and with k_closest also
# at 5 waves (lib/libpbrt_amd_wc5.so: PBRT_CLOSEST_LDS_WAVES=5).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
[ -n "$SKIP_TESTS" ] || bash tools/gpu_r6.sh r6q tests "" "" || exit $?
for v in ${VARIANTS:-main wc5}; do
  lib=$PWD/pbrt-v4_amd/lib/libpbrt_amd.so; [ $v != main ] && lib=$PWD/pbrt-v4_amd/lib/libpbrt_amd_$v.so
  [ -f $lib ] || continue
  PBRT_AMD_LIB=$lib timeout -k 10 600 python bench.py --workload c2 --steps 5 --warmup 2 --no-cpu-baseline > $O/c2_$v.log 2>&1 || { echo "bench $v failed"; tail -3 $O/c2_$v.log; exit 3; }
  tail -1 $O/c2_$v.log > $O/c2_$v.json
  python3 -c "import json; d=json.load(open('$O/c2_$v.json')); r=d['roofline']; print('c2 $v', d['value'], r.get('mean_launch_us'))"
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

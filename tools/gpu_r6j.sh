# Round-6: shading-tangent bump tests + the suite, then the BVH builder A/B: the longest-axis
# binned SAH (default) against PBRT_AMD_BVH_SAH=3 (all three axes, 32 buckets), host-only, one
# library: C4 / C3 / C2 bench lines and film hashes per builder.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6j
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
timeout -k 10 600 python -u -m pytest tests/test_shading_tangents.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -s > $O/new.log 2>&1; rc=$?
grep -E "tangents \(|passed|failed" $O/new.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r6.sh r6j tests "" "" || exit $?
for w in c4 c3 c2; do
  for sah in 0 3; do
    PBRT_AMD_BVH_SAH=$sah timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_sah$sah.log 2>&1 || { echo "bench $w $sah failed"; tail -3 $O/${w}_sah$sah.log; exit 3; }
    tail -1 $O/${w}_sah$sah.log > $O/${w}_sah$sah.json
    python3 -c "import json; d=json.load(open('$O/${w}_sah$sah.json')); r=d['roofline']; print('$w sah$sah', d['value'], r.get('mean_launch_us'))"
    hw=$w; [ "$w" = c2 ] && hw=cornell
    PBRT_AMD_BVH_SAH=$sah timeout -k 10 300 python tools/film_hash.py $hw > $O/hash_${w}_sah$sah.log 2>&1 || { echo "hash failed"; tail -3 $O/hash_${w}_sah$sah.log; exit 3; }
    tail -1 $O/hash_${w}_sah$sah.log
  done
done

# Round-6: spatial-split BVH (PBRT_AMD_BVH_SBVH=1) -- the -m gpu suite under it (oracle parity
# with duplicated leaf references), then C2 / C3 / C4 bench lines and film hashes with and without.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
PBRT_AMD_BVH_SBVH=1 bash tools/gpu_r6.sh r6l tests "" "" || exit $?
for w in c2 c3 c4; do
  for sb in 0 1; do
    PBRT_AMD_BVH_SBVH=$sb timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_sbvh$sb.log 2>&1 || { echo "bench $w $sb failed"; tail -3 $O/${w}_sbvh$sb.log; exit 3; }
    tail -1 $O/${w}_sbvh$sb.log > $O/${w}_sbvh$sb.json
    python3 -c "import json; d=json.load(open('$O/${w}_sbvh$sb.json')); r=d['roofline']; print('$w sbvh$sb', d['value'], r.get('mean_launch_us'))"
    hw=$w; [ "$w" = c2 ] && hw=cornell
    PBRT_AMD_BVH_SBVH=$sb timeout -k 10 300 python tools/film_hash.py $hw > $O/hash_${w}_sbvh$sb.log 2>&1 || { echo "hash failed"; tail -3 $O/hash_${w}_sbvh$sb.log; exit 3; }
    tail -1 $O/hash_${w}_sbvh$sb.log
  done
done

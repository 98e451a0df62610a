# BVH builder A/B (host-only, one library): the all-axes SAH (default) at traversal costs
# PBRT_AMD_BVH_CT = 0.5 (default), 1 and 2 against the longest-axis builder (PBRT_AMD_BVH_SAH=1),
# C2 / C3 / C4 bench lines and film hashes; then the -m gpu suite on the new default.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
bash tools/gpu_r6.sh r6k tests "" "" || exit $?
for w in c2 c3 c4; do
  for v in "sah1 PBRT_AMD_BVH_SAH=1" "ct05 PBRT_AMD_BVH_CT=0.5" "ct1 PBRT_AMD_BVH_CT=1" "ct2 PBRT_AMD_BVH_CT=2"; do
    set -- $v
    tag=$1; env=$2
    env $env timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_$tag.log 2>&1 || { echo "bench $w $tag failed"; tail -3 $O/${w}_$tag.log; exit 3; }
    tail -1 $O/${w}_$tag.log > $O/${w}_$tag.json
    python3 -c "import json; d=json.load(open('$O/${w}_$tag.json')); r=d['roofline']; print('$w $tag', d['value'], r.get('mean_launch_us'))"
  done
done

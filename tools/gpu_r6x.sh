# Round-6: BVH8 node order below the top levels (PBRT_AMD_BVH_DFS=k: depth-first child groups
# under depth k+1, an experiment since round 4) on C4 / C3 with the round-6 builder.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6x
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for w in c4 c3; do
  for d in 0 2 4; do
    if [ $d = 0 ]; then e=""; else e="PBRT_AMD_BVH_DFS=$d"; fi
    env $e timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_dfs$d.log 2>&1 || { echo "bench $w $d failed"; tail -3 $O/${w}_dfs$d.log; exit 3; }
    tail -1 $O/${w}_dfs$d.log > $O/${w}_dfs$d.json
    python3 -c "import json; d=json.load(open('$O/${w}_dfs$d.json')); print('$w dfs $d', d['value'], d['roofline'].get('mean_launch_us'))"
  done
done

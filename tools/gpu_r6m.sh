# Round-6: BVH leaf policy A/B -- PBRT_AMD_BVH_PAIR=1 (two-triangle nodes face the SAH leaf test)
# against the default, C2 / C3 / C4 bench lines and film hashes; then the GPU parity test file
# under it.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for w in c2 c3 c4; do
  for pr in 0 1; do
    PBRT_AMD_BVH_PAIR=$pr timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_pair$pr.log 2>&1 || { echo "bench $w $pr failed"; tail -3 $O/${w}_pair$pr.log; exit 3; }
    tail -1 $O/${w}_pair$pr.log > $O/${w}_pair$pr.json
    python3 -c "import json; d=json.load(open('$O/${w}_pair$pr.json')); r=d['roofline']; print('$w pair$pr', d['value'], r.get('mean_launch_us'))"
    hw=$w; [ "$w" = c2 ] && hw=cornell
    PBRT_AMD_BVH_PAIR=$pr timeout -k 10 300 python tools/film_hash.py $hw > $O/hash_${w}_pair$pr.log 2>&1 || { echo "hash failed"; tail -3 $O/hash_${w}_pair$pr.log; exit 3; }
    tail -1 $O/hash_${w}_pair$pr.log
  done
done
PBRT_AMD_BVH_PAIR=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/parity.log 2>&1; echo "parity rc=$?"; tail -2 $O/parity.log

# C4 ray-bin key A/B: bash tools/gpu_r6_c4ab.sh TAG "MODES"  (PBRT_AMD_RAY_BIN_KEY values)
# One bench line and one film hash per mode; films must hash the same (binning never enters a
# path's arithmetic).  Output under gpurun_out/TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; MODES=$2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for m in $MODES; do
  PBRT_AMD_RAY_BIN_KEY=$m timeout -k 10 600 python bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_key$m.log 2>&1 || { echo "bench key $m failed"; tail -5 $O/c4_key$m.log; exit 3; }
  tail -1 $O/c4_key$m.log > $O/c4_key$m.json
  python3 -c "import json,sys; d=json.load(open('$O/c4_key$m.json')); r=d['roofline']; print('key $m', d['value'], r.get('mean_launch_us'), r.get('rays_per_launch'))"
  PBRT_AMD_RAY_BIN_KEY=$m timeout -k 10 300 python tools/film_hash.py c4 > $O/hash_key$m.log 2>&1 || { echo "hash key $m failed"; tail -5 $O/hash_key$m.log; exit 3; }
  tail -1 $O/hash_key$m.log
done

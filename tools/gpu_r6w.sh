# Round-6: grid cap of the device-sized queue kernels (k_escaped / k_emissive: PBRT_AMD_EMIT_GRID,
# default 256 blocks) on C3 / C4, bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6w
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
for w in c3 c4; do
  for g in 256 1024 4096; do
    PBRT_AMD_EMIT_GRID=$g timeout -k 10 600 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/${w}_g$g.log 2>&1 || { echo "bench $w $g failed"; tail -3 $O/${w}_g$g.log; exit 3; }
    tail -1 $O/${w}_g$g.log > $O/${w}_g$g.json
    python3 -c "import json; d=json.load(open('$O/${w}_g$g.json')); print('$w grid $g', d['value'], d['ms_per_step'])"
  done
done

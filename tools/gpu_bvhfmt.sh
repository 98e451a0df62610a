# BVH node formats on C3 and C4: parity tests of both formats, then bench lines per format.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -k "bvh or c4 or c3" > gpurun_out/pytest_fmt.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_fmt.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
export PBRT_C4_DIR=/tmp/c4scene
for w in c3 c4; do
  for f in wide compressed; do
    PBRT_AMD_BVH=$f timeout -k 10 300 python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${w}_$f.log 2>&1 || { echo "bench $w $f failed"; tail -5 gpurun_out/bench_${w}_$f.log; exit 3; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${w}_$f.log').read().strip().splitlines()[-1]); print('$w', '$f', d['value'], d['roofline']['mean_launch_us'])"
  done
done

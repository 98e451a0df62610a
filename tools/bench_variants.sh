# Run bench.py once per library variant (lib/exp_*.so) on the GPU box.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_*.so; do
  PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/var.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/var.log; exit 3; }
  python3 -c "import json; d=json.loads(open('gpurun_out/var.log').read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"
done

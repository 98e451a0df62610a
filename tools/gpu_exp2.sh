set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_base.so; do
  for sc in cornell c3 c5; do
    PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 python tools/film_hash.py $sc > gpurun_out/var/hash.log 2>&1 || { echo "$lib hash failed"; tail -3 gpurun_out/var/hash.log; exit 3; }
    echo "$(basename $lib) $(tail -1 gpurun_out/var/hash.log)"
  done
done
b() { timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/var/b.log 2>&1 || { echo "bench $* failed"; tail -3 gpurun_out/var/b.log; exit 3; }
      python3 -c "import json; d=json.loads(open('gpurun_out/var/b.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"; }
echo "default"; b
echo "serial emit grid 8192"; PBRT_AMD_EMIT_SERIAL=1 PBRT_AMD_EMIT_GRID=8192 b
echo "side emit grid 64"; PBRT_AMD_EMIT_GRID=64 b
echo "side emit grid 2048"; PBRT_AMD_EMIT_GRID=2048 b
echo "c3 default"; b --workload c3 --steps 2 --warmup 1
echo "c3 base"; PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/exp_base.so b --workload c3 --steps 2 --warmup 1
echo "c5 default"; b --workload c5 --spp 128 --steps 2 --warmup 1
echo "c5 base"; PBRT_AMD_LIB=$PWD/pbrt-v4_amd/lib/exp_base.so b --workload c5 --spp 128 --steps 2 --warmup 1
timeout -k 10 200 python tools/sections.py > gpurun_out/sections.log 2>&1; echo "sections rc=$?"; tail -12 gpurun_out/sections.log

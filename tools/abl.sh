# Kernel-trace of one C2 render (tools/render_once.py) per library variant lib/exp_*.so, plus
# the default library: per-launch durations of the main kernels (tools/ktrace.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_*.so; do
  [ -f "$lib" ] || continue
  n=$(basename $lib .so)
  PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/abl/$n -o run --output-format csv -- python3 tools/render_once.py ${SPP:-16} > gpurun_out/abl/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abl/$n.log; exit 3; }
  echo "== $n"; python3 tools/ktrace.py gpurun_out/abl/$n k_shade k_closest k_shadow k_camera
done

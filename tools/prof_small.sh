# Kernel trace of one small render (floor-latency experiment)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/profs -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --xres ${XRES:-320} --yres ${YRES:-180} --spp ${SPP:-4} > gpurun_out/profs.log 2>&1 || { tail -5 gpurun_out/profs.log; exit 4; }
echo ok

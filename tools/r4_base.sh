#!/bin/bash
# Round-4 baseline on the GPU box (tools only): full GPU suite + smoke + C2 bench, then a
# rocprofv3 kernel summary of C2.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
bash tools/gpu_suite.sh r4base || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_r4base -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_r4base.log 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc

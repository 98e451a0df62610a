set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/sections.py > gpurun_out/sections.log 2>&1; echo "sections rc=$?"; cat gpurun_out/sections.log | tail -14

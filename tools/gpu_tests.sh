#!/bin/bash
# Selected GPU tests (tools only): bash tools/gpu_tests.sh TAG "pytest args"; stops at a failure.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu $2 > gpurun_out/tests_$1.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|parity|Error|passed|failed" gpurun_out/tests_$1.log | tail -30
exit $rc

#!/bin/bash
# Image-light volumetric GPU tests with the queue-hole diagnostic on (tools only): device printf
# names every queue slot a stage counted but never wrote.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
PBRT_AMD_QUEUE_CHECK=1 timeout -k 10 400 python -u -m pytest -s -v --timeout 150 --timeout-method thread \
    tests/test_envlight.py -m gpu -p no:cacheprovider > gpurun_out/qcheck.log 2>&1
rc=$?
echo "rc=$rc holes=$(grep -c 'queue hole' gpurun_out/qcheck.log)"
grep -m 20 -E "queue hole|PASSED|FAILED" gpurun_out/qcheck.log
exit $rc

#!/bin/bash
# Round-4 GPU verification of the volumetric-kernel fix (tools only): the queue-hole regression
# test first (stops at its first failure), then the image-light, shape and media GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T="python -u -m pytest -x -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 300 $T tests/test_envlight.py -k no_holes > gpurun_out/v4_holes.log 2>&1
rc=$?; echo "holes rc=$rc"; grep -E "PASSED|FAILED|queue hole|Error" gpurun_out/v4_holes.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $T tests/test_envlight.py tests/test_shapes.py tests/test_bilinear.py tests/test_gpu_media.py tests/test_gpu_layered.py > gpurun_out/v4_vol.log 2>&1
rc=$?; echo "vol rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/v4_vol.log | tail -5
exit $rc

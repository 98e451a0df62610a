# GPU layered-material parity tests (k_vlayered), then the whole GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layered.py -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_layered.log 2>&1; rc=$?
echo "layered pytest rc=$rc"; grep -E "within|PASS|FAIL|Error|^E " gpurun_out/pytest_layered.log | tail -30
if [ "$1" = "all" ] && [ $rc -le 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_layered.py > gpurun_out/pytest_gpu.log 2>&1; echo "gpu pytest rc=$?"; tail -3 gpurun_out/pytest_gpu.log
fi
exit $rc

# every GPU test, verbose log under gpurun_out/tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tests
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/tests/pytest_gpu.log 2>&1; rc=$?
echo "gpu pytest rc=$rc"; grep -E "FAILED|Error|passed|failed|vs libm|C4 full" gpurun_out/tests/pytest_gpu.log | tail -12
exit $rc

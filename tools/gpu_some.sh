# selected GPU tests: bash tools/gpu_some.sh <pytest -k expression>
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/some
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "$1" > gpurun_out/some/pytest.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "FAILED|^E |passed|failed" gpurun_out/some/pytest.log | tail -12
exit $rc

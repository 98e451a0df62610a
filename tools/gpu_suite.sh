#!/bin/bash
# Full GPU suite + smoke + a short C2 bench (tools only); stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
tag=${1:-run}
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests \
    > gpurun_out/suite_$tag.log 2>&1
rc=$?; echo "suite rc=$rc"; grep -E "passed|failed" gpurun_out/suite_$tag.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/suite_$tag.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_$tag.json
exit $rc

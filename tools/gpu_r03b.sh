# GPU tests, then C2 / C3 (auto and forced-wide) / C4 / C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest_gpu.log 2>&1; rc=$?
echo "gpu pytest rc=$rc"; tail -3 gpurun_out/r03b/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run() { name=$1; shift; timeout -k 10 400 python bench.py "$@" > gpurun_out/r03b/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/r03b/$name.log; exit 3; }; echo "$name $(tail -1 gpurun_out/r03b/$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["mean_launch_us"], (d.get("cpu_baseline") or {}).get("value"))')"; }
run c2
run c3 --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
PBRT_AMD_BVH=wide run c3wide --workload c3 --steps 2 --warmup 1 --no-cpu-baseline
export PBRT_C4_DIR=/tmp/c4scene
run c4 --workload c4 --steps 2 --warmup 1 --no-cpu-baseline
run c5 --workload c5 --steps 2 --warmup 1 --no-cpu-baseline

set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mp in 262144 524288 1048576 2097152 4194304; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --max-paths $mp > gpurun_out/sweep_$mp.log 2>&1 || { echo "fail $mp"; tail -5 gpurun_out/sweep_$mp.log; exit 3; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep_$mp.log').read().strip().splitlines()[-1]); print($mp, d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"
done

set -o pipefail
cd $GRAFT_REPO_ROOT
for w in "--workload c3 --steps 2 --warmup 1" "--workload c5 --spp 128 --steps 2 --warmup 1" "--workload c4 --steps 1 --warmup 1"; do
  BENCH_ARGS="$w" bash tools/bench_variants.sh || exit 3
done

# A/B of an environment switch on the default library: film hashes and bench lines with and
# without $AB_ENV (e.g. AB_ENV=PBRT_AMD_NO_LEAN=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for sc in ${FILM_SCENES:-cornell c3}; do
  timeout -k 10 120 python tools/film_hash.py $sc > gpurun_out/var/h.log 2>&1 || { tail -3 gpurun_out/var/h.log; exit 3; }; echo "A $(tail -1 gpurun_out/var/h.log)"
  env $AB_ENV timeout -k 10 120 python tools/film_hash.py $sc > gpurun_out/var/h.log 2>&1 || { tail -3 gpurun_out/var/h.log; exit 3; }; echo "B $(tail -1 gpurun_out/var/h.log)"
done
b() { timeout -k 10 200 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/var/b.log 2>&1 || { echo "bench failed"; tail -3 gpurun_out/var/b.log; exit 3; }
      python3 -c "import json; d=json.loads(open('gpurun_out/var/b.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['mean_launch_us'])"; }
for r in 1 2; do echo "A"; b; echo "B $AB_ENV"; env $AB_ENV bash -c "$(declare -f b); b"; done

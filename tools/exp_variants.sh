# kernel-time of build variants lib/libpbrt_amd_<v>.so on a short bench (timing experiments)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
W=${W:-c5}; SPP=${SPP:-16}
for lib in "$@"; do
  PBRT_AMD_LIB=$GRAFT_REPO_ROOT/pbrt-v4_amd/lib/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/exp_$lib -o run --output-format csv -- python3 bench.py --workload $W --spp $SPP --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/exp_$lib.log 2>&1 || exit 4
  echo "== $lib"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/exp_$lib/run_kernel_stats.csv')):
    if 'rocclr' not in r['Name']: print(f\"{r['Name'].split('(')[0][-28:]:30s} {float(r['AverageNs'])/1000:9.1f} us x{r['Calls']}\")
"
done

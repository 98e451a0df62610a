# Round profile set for the C2 headline (TAG=r02 by default): the bench line, the rocprofv3
# kernel-trace summary of the same command, the k_closest HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes, each its own run) and the traversal work per ray (profiling build).  Outputs go to
# gpurun_out/round/; copy what is judged into profiles/.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r02}
O=gpurun_out/round
rm -rf $O; mkdir -p $O/pmc
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/${TAG}_c2_bench.log 2>&1 || { tail -5 $O/${TAG}_c2_bench.log; exit 3; }
tail -1 $O/${TAG}_c2_bench.log > $O/${TAG}_c2_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 3; }
cp $(find $O/prof -name "run_kernel_stats.csv" | head -1) $O/${TAG}_c2_kernel_stats.csv
tail -1 $O/prof.log > $O/${TAG}_c2_bench_under_rocprof.json
for p in "fetch FETCH_SIZE" "write WRITE_SIZE"; do
  set -- $p
  timeout -s KILL 120 rocprofv3 --pmc $2 -d $GRAFT_REPO_ROOT/$O/pmc/$1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc/$1.log 2>&1 || { echo "pmc $1 failed"; tail -5 $O/pmc/$1.log; exit 3; }
done
for p in "sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  set -- $p
  n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$O/pmc/$n -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc/$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc/$n.log; exit 3; }
done
# the k_closest record after the SQ passes, so it carries the VALU compute roof
python3 tools/closest_pmc_json.py $O/pmc $O/${TAG}_c2_closest_pmc.json ${HEAD_SHA:+--head $HEAD_SHA} > /dev/null
python3 tools/pmc_summary.py $O/pmc --json $O/${TAG}_c2_pmc_per_kernel.json > /dev/null
python3 tools/pmc_brief.py $O/${TAG}_c2_pmc_per_kernel.json
timeout -k 10 200 python tools/trav_stats.py c2 --json $O/${TAG}_c2_trav_stats.json > $O/trav.log 2>&1 || { tail -5 $O/trav.log; exit 3; }
python3 tools/kstats.py $O/prof
cut -c1-400 $O/${TAG}_c2_bench.json
cat $O/${TAG}_closest_pmc.json | head -12
cat $O/trav.log | tail -2

# Round-6: textured subsurface + the suite, then C3's SQ counter passes (what bounds its
# k_closest: instruction mix, VALU issue and wait shares per wave) beside its traffic record.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6i
mkdir -p $O/sq
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_subsurface.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -s > $O/new.log 2>&1; rc=$?
grep -E "subsurface \(|passed|failed" $O/new.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/gpu_r6.sh r6i tests "" "" || exit $?
for p in "sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE"; do
  set -- $p
  n=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $GRAFT_REPO_ROOT/$O/sq/$n -o run --output-format csv -- python3 bench.py --workload c3 --steps 1 --warmup 1 --no-cpu-baseline > $O/sq/$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/sq/$n.log; exit 3; }
done
mkdir -p $O/sqx
for n in sq1 sq2; do f=$(find $O/sq/$n -name "*counter_collection.csv" | head -1); mkdir -p $O/sqx/$n; cp $f $O/sqx/$n/run_counter_collection.csv; done
python3 tools/pmc_summary.py $O/sqx --json $O/c3_pmc_per_kernel.json > /dev/null && python3 tools/pmc_brief.py $O/c3_pmc_per_kernel.json

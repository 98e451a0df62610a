# Round-6 final records: the -m gpu suite, the C2 bench line with its CPU baseline, C3 / C4 / C5
# bench lines, a C2 rocprofv3 kernel-trace summary, then the C2 k_closest PMC passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp PBRT_C4_DIR=/tmp/c4scene
bash tools/gpu_r6.sh r6r tests "" "" || exit $?
timeout -k 10 900 python bench.py > $O/bench_c2_full.log 2>&1 || { echo "bench c2 full failed"; tail -5 $O/bench_c2_full.log; exit 3; }
tail -1 $O/bench_c2_full.log > $O/bench_c2_full.json; cut -c1-300 $O/bench_c2_full.json
bash tools/gpu_r6.sh r6r - "c3 c4 c5" c2 || exit $?
bash tools/gpu_r6_pmc.sh r6r c2 || exit $?

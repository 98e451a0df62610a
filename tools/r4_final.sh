#!/bin/bash
# Round-4 measurement set (tools only): C2 kernel summary, per-depth queue counts, the emission
# stage serial vs beside the material stage, C4 bench + kernel summary, and C4 k_closest's HBM
# traffic (FETCH_SIZE / WRITE_SIZE / TCC hit-miss passes, each its own run).  Outputs under
# gpurun_out/r4f/; stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r4f
mkdir -p $O/pmc
export TMPDIR=/tmp
step() { echo "== $1"; }
step c2prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $O/c2_prof.log 2>&1 || { tail -5 $O/c2_prof.log; exit 3; }
python3 tools/kstats.py $O/prof_c2 | head -12
step counts
timeout -k 10 120 python3 -u tools/emit_counts.py > $O/emit_counts.txt 2>&1 || { tail -5 $O/emit_counts.txt; exit 3; }
cat $O/emit_counts.txt
step emit_serial
PBRT_AMD_EMIT_SERIAL=1 timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/c2_emit_serial.json 2>&1 || { tail -5 $O/c2_emit_serial.json; exit 3; }
tail -c 300 $O/c2_emit_serial.json | head -c 200; echo
step c4bench
timeout -k 10 500 python3 bench.py --workload c4 --steps 3 --warmup 1 > $O/c4_bench.json 2> $O/c4_bench.err || { tail -5 $O/c4_bench.err; exit 3; }
head -c 300 $O/c4_bench.json; echo
step c4prof
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/c4_prof.log 2>&1 || { tail -5 $O/c4_prof.log; exit 3; }
python3 tools/kstats.py $O/prof_c4 | head -12
for p in "fetch FETCH_SIZE" "write WRITE_SIZE" "tcc TCC_HIT_sum TCC_MISS_sum"; do
  set -- $p
  n=$1; shift
  step "pmc $n"
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d $PWD/$O/pmc/$n -o run --output-format csv -- python3 bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc/$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc/$n.log; exit 3; }
done
python3 tools/c4_pmc_json.py $O/pmc $O/c4_bench.json $O/r04_c4_closest_pmc.json "$(cat .git_head 2>/dev/null || echo r4)" && cat $O/r04_c4_closest_pmc.json | head -20

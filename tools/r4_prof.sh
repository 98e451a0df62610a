#!/bin/bash
# Round-4 profiling build runs (tools only): k_shade_diffuse section cycles on C2, traversal work
# per ray on C2 and C4.  Needs lib/libpbrt_amd_prof.so (make -C pbrt-v4_amd prof).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/sections.py > gpurun_out/sections_c2.txt 2>&1; rc=$?; echo "sections rc=$rc"; cat gpurun_out/sections_c2.txt | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/trav_stats.py c2 --json gpurun_out/r04_c2_trav_stats.json > gpurun_out/trav_c2.txt 2>&1; rc=$?; echo "trav c2 rc=$rc"; tail -3 gpurun_out/trav_c2.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/trav_stats.py c4 --json gpurun_out/r04_c4_trav_stats.json > gpurun_out/trav_c4.txt 2>&1; rc=$?; echo "trav c4 rc=$rc"; tail -3 gpurun_out/trav_c4.txt
exit $rc

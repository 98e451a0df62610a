#!/bin/bash
# A/B of library variants (tools only): film hash of each (bit-identity), then bench lines.
# Usage: bash tools/ab.sh "<film_hash args>" ; BENCH_ARGS / PROF as in bench_variants.sh
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/var
export TMPDIR=/tmp
for lib in pbrt-v4_amd/lib/libpbrt_amd.so pbrt-v4_amd/lib/exp_*.so; do
  [ -f "$lib" ] || continue
  PBRT_AMD_LIB=$PWD/$lib timeout -k 10 120 python -u tools/film_hash.py ${HASH_ARGS:-} > gpurun_out/var/hash_$(basename $lib .so).txt 2>&1 || { echo "hash $lib failed"; tail -3 gpurun_out/var/hash_$(basename $lib .so).txt; exit 3; }
  echo "$(basename $lib .so): $(tail -1 gpurun_out/var/hash_$(basename $lib .so).txt)"
done
bash tools/bench_variants.sh

#!/bin/bash
# Cost of the correctly rounded surface kernels (tools only): C2 and C4 benches with the build
# the scene selects and with PBRT_AMD_CR_MATH=1 forced.  Outputs gpurun_out/cr_*.json.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in c2 c4; do
  for cr in 0 1; do
    PBRT_AMD_CR_MATH=$cr timeout -k 10 400 python3 -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/cr_${w}_$cr.json 2> gpurun_out/cr_${w}_$cr.err || { tail -5 gpurun_out/cr_${w}_$cr.err; exit 3; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/cr_${w}_$cr.json')); print('$w cr=$cr', d['value'], d['ms_per_step'])"
  done
done

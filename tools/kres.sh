#!/bin/bash
# Per-kernel resource usage (VGPRs, spills, scratch, LDS, occupancy) of the gfx950 build.
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
  -I/root/repo/pbrt-v4_amd/csrc -c /root/repo/pbrt-v4_amd/csrc/kernels/wavefront.hip -o /tmp/wf.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re,sys
cur=None
for line in sys.stdin:
    m=re.search(r"remark: (.*?) \[-Rpass",line)
    if not m: continue
    t=m.group(1).strip()
    if t.startswith("Function Name:"):
        cur=re.sub(r"_ZN8pbrt_amd\d+(k_\w+?)E.*",r"\1",t.split(":")[1].strip()); print("\n"+cur,end=": ")
    elif any(t.startswith(k) for k in ("VGPRs:","AGPRs","ScratchSize","Occupancy","SGPRs Spill","VGPRs Spill","LDS Size")):
        print(t.replace(" [bytes/lane]","").replace(" [bytes/block]","").replace(" [waves/SIMD]",""),end="; ")
print()'

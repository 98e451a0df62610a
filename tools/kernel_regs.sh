#!/bin/bash
# Per-kernel register / spill / LDS usage of a built HIP object (tools only):
#   bash tools/kernel_regs.sh pbrt-v4_amd/build/kernels_wavefront.o [name-regex]
B=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$t/fb "$1" $t/o.tmp
$B/clang-offload-bundler --unbundle --type=o --input=$t/fb --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/co
$B/llvm-readelf --notes $t/co > $t/notes.txt
python3 - "$t/notes.txt" "${2:-.}" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for blk in txt.split("  - .agpr_count")[1:]:
    def g(k):
        m = re.search(r"\.%s:\s+(\S+)" % k, blk)
        return m.group(1) if m else "?"
    name = g("name")
    if re.search(sys.argv[2], name):
        print("%-80s vgpr %4s sgpr %4s spill %3s lds %6s" % (name[:80], g("vgpr_count"), g("sgpr_count"),
                                                           g("vgpr_spill_count"), g("group_segment_fixed_size")))
PY
rm -rf $t

#!/bin/bash
# Build experimental variants of the library: tools/variants.sh NAME "-DFLAG=..." [NAME2 "..."]
# -> pbrt-v4_amd/lib/exp_NAME.so (same host objects, kernels recompiled with the flags)
set -e
cd /root/repo/pbrt-v4_amd
make -s -j8 all
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Icsrc -Wno-unused-result $flags \
     -c csrc/kernels/wavefront.hip -o build/exp_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/exp_$name.so build/host_*.o build/exp_$name.o build/capi.o
  echo "built lib/exp_$name.so ($flags)"
done

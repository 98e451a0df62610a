#!/bin/bash
# Build experimental variants of the library: tools/variants.sh NAME "-DFLAG=..." [NAME2 "..."]
# -> pbrt-v4_amd/lib/exp_NAME.so (same host objects, both kernel files recompiled with the flags)
set -e
cd /root/repo/pbrt-v4_amd
make -s -j8 all
rm -f lib/exp_*.so
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  for k in wavefront volpath; do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Icsrc -Wno-unused-result $flags \
       -c csrc/kernels/$k.hip -o build/exp_${name}_$k.o &
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/exp_$name.so build/host_*.o build/exp_${name}_wavefront.o \
     build/exp_${name}_volpath.o build/capi.o
  echo "built lib/exp_$name.so ($flags)"
done

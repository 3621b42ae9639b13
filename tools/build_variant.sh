#!/bin/bash
# Build an A/B variant of libdprf.so with extra compiler flags: tools/build_variant.sh <name> <flags...>
# -> build/ab/libdprf_<name>.so (run on the CPU side; the .so travels to the GPU box).
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/build/ab/$N
mkdir -p $O
for f in dprf_host.cpp dprf_kernels.hip dprf_kernels_r6.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c $R/dprf_amd/csrc/$f -o $O/${f%.*}.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/build/ab/libdprf_$N.so $O/*.o
echo $R/build/ab/libdprf_$N.so

#!/bin/bash
# Build an A/B variant of libdprf.so with extra compiler flags: tools/build_variant.sh <name> <flags...>
# -> build/ab/libdprf_<name>.so (run on the CPU side; the .so travels to the GPU box).  Goes through the
# library's Makefile, so the per-object scheduler flags apply; override them through the environment
# (make's ?= variables), e.g. SCHED_R6= tools/build_variant.sh r6_default
set -e
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/build/ab/$N
mkdir -p $O
make -s -C $R/dprf_amd/csrc -j4 OUT=$R/build/ab/libdprf_$N.so OBJDIR=$O EXTRA="$*"
echo $R/build/ab/libdprf_$N.so

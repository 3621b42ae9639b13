#!/bin/bash
# -falign-loops=64 over every kernel object vs the in-tree build, all bench legs, two alternating reps (round 6).
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  timeout -k 5 280 python bench.py --cpu-seconds 0 --no-cluster > gpurun_out/ab/all_cur_$rep.json
  DPRF_LIB=$PWD/build/ab/libdprf_al64.so timeout -k 5 280 python bench.py --cpu-seconds 0 --no-cluster > gpurun_out/ab/all_al64_$rep.json
done

#!/bin/bash
# second look at ODF on two streams: five alternating pairs of 8-step runs
set -e
mkdir -p gpurun_out/ab
for rep in 1 2 3 4 5; do
  timeout -k 5 150 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 8 > gpurun_out/ab/ks1b_odt_$rep.json 2>/dev/null
  DPRF_LIB=$PWD/build/ab/libdprf_ks2.so timeout -k 5 150 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 8 > gpurun_out/ab/ks2b_odt_$rep.json 2>/dev/null
done

#!/bin/bash
# R6: CBC xor + first AddRoundKey as one v_bitop3 per word (build/ab/libdprf_x3.so) vs the in-tree build (round 6):
# the R6 GPU tests on the variant first, then alternating bench runs.
set -e
mkdir -p gpurun_out/ab
DPRF_LIB=$PWD/build/ab/libdprf_x3.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "r6" > gpurun_out/ab/x3_tests.log 2>&1
tail -1 gpurun_out/ab/x3_tests.log
for rep in 1 2 3; do
  timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6cur_$rep.json 2>/dev/null
  DPRF_LIB=$PWD/build/ab/libdprf_x3.so timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6x3_$rep.json 2>/dev/null
done

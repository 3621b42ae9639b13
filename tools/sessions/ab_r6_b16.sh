#!/bin/bash
# R6: base >> 16 once per AES block (build/ab/libdprf_b16.so) vs the in-tree build (round 6): the whole GPU suite on the variant
# first, then alternating bench runs.
set -e
mkdir -p gpurun_out/ab
DPRF_LIB=$PWD/build/ab/libdprf_b16.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/b16_tests.log 2>&1
tail -1 gpurun_out/ab/b16_tests.log
for rep in 1 2 3; do
  timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6x3c_$rep.json 2>/dev/null
  DPRF_LIB=$PWD/build/ab/libdprf_b16.so timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6b16_$rep.json 2>/dev/null
done

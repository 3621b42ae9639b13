#!/bin/bash
# R6: dword-wise K store (build/ab/libdprf_sk.so) vs the in-tree build (round 6): the whole GPU suite on the variant
# first, then alternating bench runs.
set -e
mkdir -p gpurun_out/ab
DPRF_LIB=$PWD/build/ab/libdprf_sk.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/sk_tests.log 2>&1
tail -1 gpurun_out/ab/sk_tests.log
for rep in 1 2 3; do
  timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6x3b_$rep.json 2>/dev/null
  DPRF_LIB=$PWD/build/ab/libdprf_sk.so timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --warmup 1 > gpurun_out/ab/r6sk_$rep.json 2>/dev/null
done

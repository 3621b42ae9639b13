#!/bin/bash
# PDF R5 launches alternating two streams per device (build/ab/libdprf_r5s2.so, -DDPRF_R5_STREAMS=2) vs one
# (in-tree), round 6: range-mode bench leg and the symbol window, alternating; R5 GPU tests on the variant first.
set -e
mkdir -p gpurun_out/ab
DPRF_LIB=$PWD/build/ab/libdprf_r5s2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "r5 or symbol or stop" > gpurun_out/ab/r5s_tests.log 2>&1
tail -1 gpurun_out/ab/r5s_tests.log
for rep in 1 2 3; do
  timeout -k 5 150 python bench.py --workload pdf_r5 --no-side --cpu-seconds 0 --steps 5 > gpurun_out/ab/r5s1_$rep.json 2>/dev/null
  DPRF_LIB=$PWD/build/ab/libdprf_r5s2.so timeout -k 5 150 python bench.py --workload pdf_r5 --no-side --cpu-seconds 0 --steps 5 > gpurun_out/ab/r5s2_$rep.json 2>/dev/null
done
timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5 > gpurun_out/ab/r5s1_sym.jsonl 2>/dev/null
DPRF_LIB=$PWD/build/ab/libdprf_r5s2.so timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5 > gpurun_out/ab/r5s2_sym.jsonl 2>/dev/null

#!/bin/bash
# R5 list launches of short candidates on the one-block kernels (round 6): GPU tests, then the R5 symbol-window rate
# (tools/bench_symbols.py) with the r06f library and the in-tree one, alternating.
set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_r5_list.py tests/test_symbols.py tests/test_planted_edges.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "r5 or symbol or pdf" > gpurun_out/ab/r5l_tests.log 2>&1
tail -1 gpurun_out/ab/r5l_tests.log
for rep in 1 2; do
  DPRF_LIB=$PWD/build/ab/libdprf_r06f.so timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5 > gpurun_out/ab/r5l_old_$rep.json 2>/dev/null
  timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5 > gpurun_out/ab/r5l_new_$rep.json 2>/dev/null
done

#!/bin/bash
# R6 A/B on one box: in-tree build (tests first, under a short timeout) vs build/ab/libdprf_base.so, and a
# -DDPRF_R6_TIMING build's per-wave split.
set -e
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py tests/test_full_size.py -m gpu -x -q --timeout 60 --timeout-method thread -k "r6 or verdict or hitset or docs" > gpurun_out/r6_tests.log 2>&1
timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 > gpurun_out/r6_new.json
DPRF_LIB=$PWD/build/ab/libdprf_base.so timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 > gpurun_out/r6_base.json
DPRF_LIB=$PWD/build/ab/libdprf_tim.so timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > gpurun_out/r6_tim.out 2>&1

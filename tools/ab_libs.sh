#!/bin/bash
# A/B several library builds on one box for one workload: parity tests of that family under each, then
# bench.  Usage: tools/ab_libs.sh <workload> <pytest -k expr> <variant>...   (variant "base" = in-tree)
set -e
W=$1; K=$2; shift 2
for V in "$@"; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  DPRF_LIB=$L timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py -m gpu -x -q --timeout 60 --timeout-method thread -k "$K" > gpurun_out/ab_${V}_tests.log 2>&1
  for rep in 1 2; do
    DPRF_LIB=$L timeout -k 5 100 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 2 | python -c "import json,sys; d=json.load(sys.stdin); print('$V', d['value'], d['roofline']['frac'])"
  done
done

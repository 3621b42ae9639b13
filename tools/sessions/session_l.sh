#!/bin/bash
# GPU session L (round 4): R2 batches per workgroup (base = 24) with two-stream launches
set -e
DPRF_LIB=$PWD/build/ab/libdprf_r2b48.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread -k "r2" 2>&1 | tail -1
for rep in 1 2 3; do
  for V in base r2b16 r2b36 r2b48; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 120 python bench.py --workload pdf_r2 --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V', round(d['value']/1e9,3), int(r['candidates_per_launch']))"
  done
done
echo "== done $(date +%T)"

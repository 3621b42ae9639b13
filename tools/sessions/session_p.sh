#!/bin/bash
# GPU session P (round 4): PDF R6 launches alternating between two streams (DPRF_R6_STREAMS=2, a work cursor per
# stream) -- R6 parity of the variant, then alternating bench runs against the product build (one stream)
set -e
DPRF_LIB=$PWD/build/ab/libdprf_r6_2s.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" 2>&1 | tail -1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" 2>&1 | tail -1
for rep in 1 2 3; do
  for V in base r6_2s; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$rep $V', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],1), int(d['roofline']['candidates_per_launch']))"
  done
done
echo "== done $(date +%T)"

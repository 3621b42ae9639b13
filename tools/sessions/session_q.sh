#!/bin/bash
# GPU session Q (round 4): PDF R6 AES lookups of state byte 1 by v_bitop3 instead of v_perm (R6_B1_BITOP3) --
# R6 parity of the variant, then alternating bench runs against the product build
set -e
DPRF_LIB=$PWD/build/ab/libdprf_r6_b1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" 2>&1 | tail -1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" 2>&1 | tail -1
for rep in 1 2 3; do
  for V in base r6_b1; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$rep $V', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],1), int(d['roofline']['candidates_per_launch']))"
  done
done
echo "== done $(date +%T)"

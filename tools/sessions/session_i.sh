#!/bin/bash
# GPU session I (round 4): R3/R4 launch overlap -- two streams, bigger launches, both
set -e
for rep in 1 2 3; do
  for V in base r24_2s r24_2s_t200 r24_t400; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 120 python bench.py --workload pdf_r34 --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V', round(d['value']/1e6,2), round(r['kernel_avg_ms'],2), int(r['candidates_per_launch']))"
  done
done

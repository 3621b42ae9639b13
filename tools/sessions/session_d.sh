#!/bin/bash
# GPU session D (round 4): PDF R6 launch size A/B -- the drain at the end of every launch of the persistent kernel
# (tools/r6 flow simulation: 2^22 / 2^23 / 2^24 candidates per launch fill 62.2 / 63.0 / 63.5 lanes per batch).
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
for rep in 1 2 3; do
  for V in base r6_t6000; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 3 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V', round(d['value']/1e6,4), round(r['kernel_avg_ms'],1), int(r['candidates_per_launch']))"
  done
  V=r6_t6000_hi25; L=$PWD/build/ab/libdprf_$V.so
  DPRF_LIB=$L timeout -k 5 200 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 3 --batch 33554432 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V (2^25 per step)', round(d['value']/1e6,4), round(r['kernel_avg_ms'],1), int(r['candidates_per_launch']))"
done
echo "== done $(date +%T)"

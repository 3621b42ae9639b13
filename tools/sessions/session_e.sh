#!/bin/bash
# GPU session E (round 4): ODF / Office launch size A/B (the partial last generation of resident workgroups per launch)
set -e
TAG=${1:?tag}
for rep in 1 2 3; do
  for V in base odt_big; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    for W in odt office; do
      DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V $W', round(d['value']/1e6,4), round(r['kernel_avg_ms'],2), int(r['candidates_per_launch']), round(r['frac'],4))"
    done
  done
done

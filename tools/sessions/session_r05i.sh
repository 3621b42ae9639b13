#!/bin/bash
# round 5 session I: ODF KDF object under other LLVM scheduler strategies (max-memory-clause; max-ilp at 5 waves/SIMD,
# 12 B/lane of scratch, gate off) against the shipped default-strategy build: three alternating odt bench rounds
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
for rep in 1 2 3; do
  for L in base odt_max-memory-clause odt_milp5; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 5 > $O/b_${rep}_$L.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/b_${rep}_$L.json')); print('$rep $L', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],2))" | tee -a $O/summary.txt
  done
done

#!/bin/bash
# GPU session R (round 4): the ODF check kernel's byte-1 inverse-cipher lookups by v_bitop3 (ODT_B1_BITOP3) -- ODF /
# Office parity of the variant, then alternating ODF bench runs (check-kernel ms from the bench line's kernel split)
set -e
DPRF_LIB=$PWD/build/ab/libdprf_odt_b1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread -k "odt or ODT or odf" 2>&1 | tail -1
for rep in 1 2 3; do
  for V in base odt_b1; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V', round(d['value']/1e6,4), round(r['kernel_avg_ms'],2), round(d['ms_per_step'],2))"
  done
done
echo "== done $(date +%T)"

#!/bin/bash
# GPU session O (round 4): RC4 KSA identity rows 0-23 from loop-invariant input VGPRs (gen_rc4_ksa_asm.py --idregs 24)
set -e
DPRF_LIB=$PWD/build/ab/libdprf_r24_id24.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 100 --timeout-method thread -k "r2 or r3 or r4 or R3 or R4 or R2 or hitsets or verdict" 2>&1 | tail -1
for rep in 1 2 3; do
  for V in base r24_id24; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    for W in pdf_r34 pdf_r2; do
      DPRF_LIB=$L timeout -k 5 120 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V $W', round(d['value']/1e6,2), int(r['candidates_per_launch']))"
    done
  done
done
echo "== done $(date +%T)"

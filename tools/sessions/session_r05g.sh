#!/bin/bash
# round 5 session G: ODF KDF with the two PBKDF2 output blocks' SHA-1s in lockstep (ODT_KDF_PAIR, 5 waves/SIMD) vs the
# shipped kernel: ODF parity tests on the variant, then three alternating bench rounds of odt and odt_e
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
V=${1:-odtpair5}
DPRF_LIB=build/ab/libdprf_$V.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py -m gpu -k "odt or odf or verdict or hitsets or docs" > $O/tests_$V.log 2>&1; rc=$?
echo "tests $V rc=$rc $(tail -n 1 $O/tests_$V.log)" | tee -a $O/summary.txt
[ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for L in base $V; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    for W in odt odt_e; do
      DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 5 > $O/b_${rep}_${L}_$W.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('$O/b_${rep}_${L}_$W.json')); print('$rep $L $W', round(d['value']/1e6,3), round(d['roofline']['kernel_avg_ms'],2))" | tee -a $O/summary.txt
    done
  done
done

#!/bin/bash
# round 5 session H: two independent SHA-1 streams per lane -- ODF's two PBKDF2 blocks in lockstep (odtpair5,
# ODT_KDF_PAIR at 5 waves/SIMD) and two Office candidates per lane (offpair, OFFICE_KDF_PAIR) -- against the shipped
# kernels: their parity tests first, then three alternating bench rounds
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
for V in odtpair5 offpair; do
  DPRF_LIB=build/ab/libdprf_$V.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py tests/test_protocol.py -m gpu \
      -k "odt or odf or office or verdict or hitsets or docs or long or config5" > $O/tests_$V.log 2>&1; rc=$?
  echo "tests $V rc=$rc $(tail -n 1 $O/tests_$V.log)" | tee -a $O/summary.txt
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for L in base odtpair5 offpair; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    for W in odt office; do
      [ "$L" = odtpair5 ] && [ $W = office ] && continue
      [ "$L" = offpair ] && [ $W = odt ] && continue
      DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 5 > $O/b_${rep}_${L}_$W.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('$O/b_${rep}_${L}_$W.json')); print('$rep $L $W', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],2))" | tee -a $O/summary.txt
    done
  done
done

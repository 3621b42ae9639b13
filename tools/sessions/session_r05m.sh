#!/bin/bash
# round 5 session M: the --bytes KSA (S[i] pair as two byte loads / stores, full-rate selects) -- S-box probe, chain
# latency probe, R2-R4 parity tests on the product build, then three alternating bench rounds vs the shipped KSA
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
chk() { local rc=$1; if [ $rc -ge 124 ]; then echo "STOP rc=$rc" | tee -a $O/summary.txt; exit $rc; fi; }
timeout -k 10 60 build/probe/probe_bytes 4608 20 > $O/probe_bytes.log 2>&1; rc=$?
echo "probe bytes rc=$rc $(tail -n 1 $O/probe_bytes.log)" | tee -a $O/summary.txt; chk $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 build/probe/probe_bytes time 4000 > $O/latency_bytes.jsonl 2>&1; rc=$?
echo "latency bytes rc=$rc" | tee -a $O/summary.txt; chk $rc
DPRF_LIB=build/ab/libdprf_bytes.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_full_size.py -m gpu -k "verdict or hitsets or r2 or r3 or r4 or R2 or R3 or R4 or pdf" \
    > $O/tests_bytes.log 2>&1; rc=$?
echo "tests bytes rc=$rc $(tail -n 1 $O/tests_bytes.log)" | tee -a $O/summary.txt; chk $rc
[ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  for L in base bytes; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    for W in pdf_r34 pdf_r2; do
      DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 > $O/b_${rep}_${L}_$W.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('$O/b_${rep}_${L}_$W.json')); print('$rep $L $W', round(d['value']/1e6,2))" | tee -a $O/summary.txt
    done
  done
done

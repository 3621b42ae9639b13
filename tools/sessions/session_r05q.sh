#!/bin/bash
# round 5 session Q: PDF R5 runs with the run length per launch (16 for >= 16 characters, else 8) and the register
# budget of 4 waves per SIMD -- R5 parity on the candidate default, the new run tests on the variants, then three
# alternating bench rounds: shipped / v2 (16, 4 waves) / v2 with runs of 8 only / v2 at 5 waves per SIMD
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
chk() { local rc=$1; if [ $rc -ge 124 ]; then echo "STOP rc=$rc" | tee -a $O/summary.txt; exit $rc; fi; }
DPRF_LIB=build/ab/libdprf_r5v2.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_r5_runs.py tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py -m gpu -k "r5 or R5 or runs or pdf" \
    > $O/tests_r5v2.log 2>&1; rc=$?
echo "tests r5v2 rc=$rc $(tail -n 1 $O/tests_r5v2.log)" | tee -a $O/summary.txt; chk $rc
[ $rc -eq 0 ] || exit 1
for L in r5v2_p8 r5v2_w5; do
  DPRF_LIB=build/ab/libdprf_$L.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_r5_runs.py -m gpu > $O/tests_$L.log 2>&1; rc=$?
  echo "tests $L rc=$rc $(tail -n 1 $O/tests_$L.log)" | tee -a $O/summary.txt; chk $rc
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for L in base r5v2 r5v2_p8 r5v2_w5; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload pdf_r5 --no-side --cpu-seconds 0 --steps 4 > $O/b_${rep}_${L}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/b_${rep}_${L}.json')); print('$rep $L pdf_r5', round(d['value']/1e9,3), round(d['roofline']['kernel_avg_ms'],3))" | tee -a $O/summary.txt
  done
done

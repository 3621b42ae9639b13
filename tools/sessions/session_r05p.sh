#!/bin/bash
# round 5 session P: PDF R5 range mode by runs of consecutive candidates + one instantiation per candidate-word
# count (k_pdf_r5 R5_RUNS / NW) -- R5 parity tests on each variant, then three alternating bench rounds against the
# shipped build: runs (R5_PER 8), runs with R5_PER 16, runs with the register budget of 4 waves per SIMD
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
chk() { local rc=$1; if [ $rc -ge 124 ]; then echo "STOP rc=$rc" | tee -a $O/summary.txt; exit $rc; fi; }
DPRF_LIB=build/ab/libdprf_r5run.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_r5_runs.py tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py -m gpu -k "r5 or R5 or runs or pdf" \
    > $O/tests_r5run.log 2>&1; rc=$?
echo "tests r5run rc=$rc $(tail -n 1 $O/tests_r5run.log)" | tee -a $O/summary.txt; chk $rc
[ $rc -eq 0 ] || exit 1
for L in r5run16 r5run_w4; do
  DPRF_LIB=build/ab/libdprf_$L.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_r5_runs.py -m gpu > $O/tests_$L.log 2>&1; rc=$?
  echo "tests $L rc=$rc $(tail -n 1 $O/tests_$L.log)" | tee -a $O/summary.txt; chk $rc
  [ $rc -eq 0 ] || exit 1
done
for rep in 1 2 3; do
  for L in base r5run r5run16 r5run_w4; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload pdf_r5 --no-side --cpu-seconds 0 --steps 4 > $O/b_${rep}_${L}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/b_${rep}_${L}.json')); print('$rep $L pdf_r5', round(d['value']/1e9,3), round(d['roofline']['kernel_avg_ms'],3))" | tee -a $O/summary.txt
  done
done

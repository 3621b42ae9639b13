#!/bin/bash
# round 5 session L: RC4 waves of a CU at 2 or 3 different issue priorities (R24_PRIO_SPLIT, all above the key waves)
# vs one priority for all (shipped): three alternating bench rounds of pdf_r34 and pdf_r2
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
for rep in 1 2 3; do
  for L in base prio2 prio3; do
    if [ "$L" = "base" ]; then LIB=$PWD/dprf_amd/libdprf.so; else LIB=$PWD/build/ab/libdprf_$L.so; fi
    for W in pdf_r34 pdf_r2; do
      DPRF_LIB=$LIB timeout -k 10 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 > $O/b_${rep}_${L}_$W.json 2>/dev/null || exit 1
      python -c "import json; d=json.load(open('$O/b_${rep}_${L}_$W.json')); print('$rep $L $W', round(d['value']/1e6,2))" | tee -a $O/summary.txt
    done
  done
done
DPRF_LIB=build/ab/libdprf_prio3.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k verdict > $O/tests_prio3.log 2>&1
echo "tests prio3 rc=$? $(tail -n 1 $O/tests_prio3.log)" | tee -a $O/summary.txt

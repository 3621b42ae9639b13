#!/bin/bash
# round 5 session B: (1) S-box probes of the --mskor and the pre-fix --idregs (--no-m0-wait) schedules; (2) the
# chain-latency probe (base, mskor); (3) the mskor and idregs product builds against the R2-R4 parity tests; (4) three
# alternating bench rounds base / mskor / id24 on pdf_r34 and pdf_r2.  Every GPU step has its own time limit and the
# script stops at the first that times out or crashes.
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
chk() { local rc=$1; if [ $rc -ge 124 ] || [ $rc -ge 128 ]; then echo "STOP rc=$rc" | tee -a $O/summary.txt; exit $rc; fi; }
for v in mskor id24nw; do
  timeout -k 10 60 build/probe/probe_$v 4608 20 > $O/probe_$v.log 2>&1; rc=$?
  echo "probe $v rc=$rc $(tail -n 1 $O/probe_$v.log)" | tee -a $O/summary.txt; chk $rc
done
for v in base mskor; do
  timeout -k 10 120 build/probe/probe_$v time 4000 > $O/latency_$v.jsonl 2>&1; rc=$?
  echo "latency $v rc=$rc" | tee -a $O/summary.txt; chk $rc
done
for v in mskor id24; do
  DPRF_LIB=build/ab/libdprf_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_parity.py tests/test_full_size.py -m gpu -k "verdict or hitsets or r2 or r3 or r4 or R2 or R3 or R4 or pdf" \
      > $O/tests_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc $(tail -n 1 $O/tests_$v.log)" | tee -a $O/summary.txt; chk $rc
done
for rep in 1 2 3; do
  for V in base mskor id24; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    for W in pdf_r34 pdf_r2; do
      DPRF_LIB=$L timeout -k 10 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 > $O/bench_${rep}_${V}_$W.json 2>$O/bench_${rep}_${V}_$W.err; rc=$?
      chk $rc
      python -c "import json,sys; d=json.load(open('$O/bench_${rep}_${V}_$W.json')); r=d['roofline']; print('$rep $V $W', round(d['value']/1e6,2), int(r['candidates_per_launch']))" | tee -a $O/summary.txt
    done
  done
done
echo "== done $(date +%T)" | tee -a $O/summary.txt

#!/bin/bash
# round 5 session A: why the --idregs 24 KSA variant fails the R4 list-mode verdict on the MI355X.
#  1. the plain idregs library against the reference verdict tables (the round-4 failure, re-run once)
#  2. the debug builds (-DDPRF_DEBUG_R24) of base and idregs: tools/r24_dump.py traces the R3/R4 chain per pass
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/r05a
mkdir -p $O
DPRF_LIB=build/ab/libdprf_id24.so timeout -k 10 180 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu -k verdict_tables > $O/id24_verdicts.log 2>&1
echo "id24 verdict tables rc=$?" | tee -a $O/summary.txt
for v in dbg_base dbg_id24; do
  for t in pdf_testdoc_r4 pdf_synth_r3_l128_abc pdf_synth_r3_l40_cab; do
    DPRF_LIB=build/ab/libdprf_$v.so timeout -k 10 120 python -u tools/r24_dump.py $t > $O/${v}_$t.log 2>&1
    rc=$?
    echo "$v $t rc=$rc $(tail -n 1 $O/${v}_$t.log)" | tee -a $O/summary.txt
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
#  3. the R2-R4 chain latency: one R3/R4 pass (asm KSA + PRGA-2) at 1..9 one-wave workgroups per CU
timeout -k 10 120 build/probe/probe_base time 400 > $O/rc4_latency.jsonl 2>&1
echo "latency probe rc=$?" | tee -a $O/summary.txt

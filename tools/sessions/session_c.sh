#!/bin/bash
# GPU session C (round 4): PDF R6 claim A/B -- batch fill from the -DDPRF_R6_TIMING builds (base vs reserving claim),
# parity of the reserving build, alternating bench runs.  Usage on the box: tools/session_c.sh <tag>
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
for V in r6_tim r6_reserve2_tim; do
  DPRF_LIB=$PWD/build/ab/libdprf_$V.so timeout -k 10 120 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > gpurun_out/${V}_$TAG.txt 2>&1
  python3 - gpurun_out/${V}_$TAG.txt $V <<'PY'
import re, sys
b = s = w = wt = 0
for ln in open(sys.argv[1]):
    m = re.search(r"work (\d+) wait (\d+) batches (\d+) slots (\d+)", ln)
    if m:
        w += int(m.group(1)); wt += int(m.group(2)); b += int(m.group(3)); s += int(m.group(4))
print(sys.argv[2], "slots per batch %.2f" % (s / max(1, b)), "wait frac %.4f" % (wt / max(1, w + wt)), "batches", b)
PY
done
echo "== parity r6_reserve2 $(date +%T)"
DPRF_LIB=$PWD/build/ab/libdprf_r6_reserve2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" > gpurun_out/ab_r6_reserve2_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_r6_reserve2_$TAG.log; exit 1; }
tail -1 gpurun_out/ab_r6_reserve2_$TAG.log
for rep in 1 2 3; do
  for V in base r6_reserve2; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 3 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$rep $V', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],2))"
  done
done
echo "== done $(date +%T)"

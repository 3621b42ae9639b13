#!/bin/bash
# GPU session H (round 4): R2-R4 launches alternating over two streams per device (DPRF_R24_STREAMS=2) vs one
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
DPRF_LIB=$PWD/build/ab/libdprf_r24_2s.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "pdf or stop_on_first or multi_device or chunk" > gpurun_out/ab_r24_2s_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_r24_2s_$TAG.log; exit 1; }
tail -1 gpurun_out/ab_r24_2s_$TAG.log
for rep in 1 2 3; do
  for V in base r24_2s; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    for W in pdf_r34 pdf_r2 pdf_r3_40; do
      DPRF_LIB=$L timeout -k 5 120 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 4 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$rep $V $W', round(d['value']/1e6,2), round(r['kernel_avg_ms'],2), int(r['candidates_per_launch']))"
    done
  done
done
echo "== done $(date +%T)"

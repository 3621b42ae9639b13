#!/bin/bash
# Office / ODF launches alternating two streams per device (-DDPRF_KDF_STREAMS=2, build/ab/libdprf_ks2.so) vs one
# (in-tree), round 6: the next launch's KDF can start while this one's check kernel and last KDF workgroups run.
set -e
mkdir -p gpurun_out/ab
DPRF_LIB=$PWD/build/ab/libdprf_ks2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "odt or office or docx or symbol or stop" > gpurun_out/ab/ks2_tests.log 2>&1
tail -1 gpurun_out/ab/ks2_tests.log
for rep in 1 2 3; do
  for w in odt office; do
    timeout -k 5 150 python bench.py --workload $w --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/ks1_${w}_$rep.json 2>/dev/null
    DPRF_LIB=$PWD/build/ab/libdprf_ks2.so timeout -k 5 150 python bench.py --workload $w --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/ks2_${w}_$rep.json 2>/dev/null
  done
done

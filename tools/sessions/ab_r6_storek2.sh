#!/bin/bash
# R6 dword K store, second look (round 6): x3 (in-tree) / sk / x3 + -falign-loops=64 / sk + -falign-loops=64,
# alternating, then one SQ pass on x3 and sk (VALU instructions and busy cycles of the same work).
set -e
R=$PWD
mkdir -p gpurun_out/ab
B="python3 $R/bench.py --workload pdf_r6 --no-side --cpu-seconds 0"
for rep in 1 2; do
  for v in x3 sk x3al skal; do
    if [ $v = x3 ]; then L=$R/dprf_amd/libdprf.so; else L=$R/build/ab/libdprf_$v.so; fi
    DPRF_LIB=$L timeout -k 5 150 $B --steps 2 --warmup 1 > gpurun_out/ab/r6w_${v}_$rep.json 2>/dev/null
  done
done
cd /tmp && export TMPDIR=/tmp
for v in x3 sk; do
  if [ $v = x3 ]; then L=$R/dprf_amd/libdprf.so; else L=$R/build/ab/libdprf_$v.so; fi
  DPRF_LIB=$L timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/ab/pmc_$v -o sq --output-format csv -- $B --steps 1 --warmup 1 > /dev/null
done

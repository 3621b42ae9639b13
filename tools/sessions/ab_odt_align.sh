#!/bin/bash
# ODF PBKDF2 loop-offset sweep on one box (round 6): the in-tree build (loop tops 16/28 mod 64) and
# -DODT_LOOP_PAD=P, P=1..15 s_nop words before the block-1 loop (both loops move by 4P bytes), two reps, interleaved.
set -e
mkdir -p gpurun_out/ab
for rep in 1 2; do
  timeout -k 5 100 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/odt0_$rep.json 2>/dev/null
  for P in $(seq 1 15); do
    DPRF_LIB=$PWD/build/ab/libdprf_odt$P.so timeout -k 5 100 python bench.py --workload odt --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/odt${P}_$rep.json 2>/dev/null
  done
done

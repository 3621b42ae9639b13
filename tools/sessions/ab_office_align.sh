#!/bin/bash
# Office KDF loop-alignment A/B on one box (round 6): the in-tree build (50,000-iteration loop top at 60 mod 64),
# -DOFFICE_LOOP_PAD=1 (0 mod 64) and =3 (8 mod 64, where round 5's build had it), and round 5's own build/tree,
# alternating, three reps each.
set -e
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  timeout -k 5 100 python bench.py --workload office --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/cur_$rep.json
  DPRF_LIB=$PWD/build/ab/libdprf_pad1.so timeout -k 5 100 python bench.py --workload office --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/pad1_$rep.json
  DPRF_LIB=$PWD/build/ab/libdprf_pad3.so timeout -k 5 100 python bench.py --workload office --no-side --cpu-seconds 0 --steps 4 > gpurun_out/ab/pad3_$rep.json
  (cd build/ab/r05 && DPRF_LIB=$PWD/libdprf.so timeout -k 5 100 python bench.py --workload office --no-side --cpu-seconds 0 --steps 4 > ../../../gpurun_out/ab/r05_$rep.json)
done

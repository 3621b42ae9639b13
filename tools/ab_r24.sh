# A/B of R2-R4 kernel builds on one box: HEAD vs the working tree
set -e
for w in pdf_r34 pdf_r2; do
  for v in head new; do
    if [ $v = new ]; then L=""; else L=$PWD/build/ab/libdprf_$v.so; fi
    DPRF_LIB=$L timeout -k 10 200 python bench.py --workload $w --no-side --cpu-seconds 0 > gpurun_out/ab_${v}_$w.json
  done
done

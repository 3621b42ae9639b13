# A/B of R6 builds on one box
set -e
for v in r6head r6g1; do
  DPRF_LIB=$PWD/build/ab/libdprf_$v.so timeout -k 10 200 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_$v.json
done
timeout -k 10 200 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_r6g3.json

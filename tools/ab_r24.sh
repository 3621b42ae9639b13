# A/B of R2-R4 kernel builds on one box: the in-tree build vs build/ab/libdprf_<variant>.so for each variant
# named on the command line (default: head).  Usage: tools/ab_r24.sh [variant...]
set -e
VARS=${@:-head}
for w in pdf_r34 pdf_r2; do
  timeout -k 10 200 python bench.py --workload $w --no-side --cpu-seconds 0 > gpurun_out/ab_new_$w.json
  for v in $VARS; do
    DPRF_LIB=$PWD/build/ab/libdprf_$v.so timeout -k 10 200 python bench.py --workload $w --no-side --cpu-seconds 0 > gpurun_out/ab_${v}_$w.json
  done
done

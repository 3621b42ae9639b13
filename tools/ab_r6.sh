# A/B of R6 builds on one box: in-tree build vs build/ab/libdprf_<v>.so for each variant named (parity tests
# on each variant first).  Usage: tools/ab_r6.sh v1 [v2 ...]
set -e
timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_base.json
for V in "$@"; do
  L=$PWD/build/ab/libdprf_$V.so
  DPRF_LIB=$L timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py -m gpu -x -q --timeout 100 --timeout-method thread -k "r6" > gpurun_out/ab_${V}_tests.log 2>&1
  DPRF_LIB=$L timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_$V.json
done

# A/B of R6 builds on one box: in-tree build vs build/ab/libdprf_$1.so (parity tests on the variant first)
set -e
V=${1:-r6p}
L=$PWD/build/ab/libdprf_$V.so
DPRF_LIB=$L timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py -m gpu -x -q --timeout 100 --timeout-method thread -k "r6" > gpurun_out/ab_${V}_tests.log 2>&1
timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_base.json
DPRF_LIB=$L timeout -k 5 100 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 > gpurun_out/ab_$V.json

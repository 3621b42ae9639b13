#!/bin/bash
# R6 launch size A/B (the persistent kernel drains at the end of every launch): same 2^23-candidate
# steps, chunk 2^21 / 2^22 / 2^23 per launch (build/ab/libdprf_c2N.so from tools/build_variant.sh).
set -e
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py tests/test_full_size.py -m gpu -x -q --timeout 60 --timeout-method thread -k "r6 or verdict" > gpurun_out/ab_r6chunk_tests.log 2>&1
for V in c21 c22 c23; do
  for rep in 1 2; do
    DPRF_LIB=$PWD/build/ab/libdprf_$V.so timeout -k 5 120 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 --batch 8388608 | python -c "import json,sys; d=json.load(sys.stdin); print('$V', d['value'], d['roofline']['frac'], d['roofline']['candidates_per_launch'])"
  done
done

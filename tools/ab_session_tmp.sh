mkdir -p gpurun_out
ab() { W=$1; shift; for V in "$@"; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  for rep in 1 2; do DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 | python -c "import json,sys; d=json.load(sys.stdin); print('$W $V', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])"; done
done; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pdf or r24 or r34 or r2 or R4 or R3 or R2" > gpurun_out/gputests_b128.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/gputests_b128.log)"
ab pdf_r34 base r24_addtid
ab pdf_r2 base r24_addtid

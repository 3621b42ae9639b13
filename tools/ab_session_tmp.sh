mkdir -p gpurun_out
ab() { W=$1; shift; for V in "$@"; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 | python -c "import json,sys; d=json.load(sys.stdin); print('$W $V', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])" || exit 1
done; }
DPRF_LIB=$PWD/build/ab/libdprf_sb16.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread -k "r6 or R6 or pdf or families or hitsets or verdict" > gpurun_out/gputests_sb16.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/gputests_sb16.log)"
ab pdf_r6 sb0 sb16 l512 l512s0 sb0 sb16 l512 l512s0

mkdir -p gpurun_out
ab() { W=$1; shift; for V in "$@"; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 | python -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print('$W $V', d['value'], r['frac'], r['kernel_avg_ms'])" || exit 1
done; }
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_docs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "odt or families or hitsets or verdict" > gpurun_out/gputests_pre.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/gputests_pre.log)"
ab odt base prev base prev base prev

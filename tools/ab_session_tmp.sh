mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r03d.log 2>&1
echo "tests rc=$? $(tail -1 gpurun_out/gputests_r03d.log)"
ab() { W=$1; shift; for V in "$@"; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  for rep in 1 2; do DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 | python -c "import json,sys; d=json.load(sys.stdin); print('$W $V', d['value'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])"; done
done; }
ab pdf_r6 base
ab pdf_r34 base r24_late
ab pdf_r2 base r24_late
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r6lds -o lds --output-format csv -- python3 $R/bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > /dev/null
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/r6write -o write --output-format csv -- python3 $R/bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > /dev/null
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/r34lds -o lds --output-format csv -- python3 $R/bench.py --workload pdf_r34 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > /dev/null
echo done

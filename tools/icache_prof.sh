# I-cache counters for the production R4 kernel and the rc4 micro-benchmark
set -e
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/ic_prod -o p --output-format csv -- python3 $R/bench.py --workload pdf_r34 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > /dev/null
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --kernel-trace -d $R/gpurun_out/ic_micro -o p --output-format csv -- $R/tools/rc4_bench 16384 1 > /dev/null
cd $R && timeout -k 10 60 ./tools/rc4_bench 65536 3 > gpurun_out/rc4_bench.txt

#!/bin/bash
# k_spell_symbols with coalesced slot stores and no digit array (in-tree) vs the first version (build/ab/libdprf_sp0.so):
# symbol and R5-list GPU tests, then tools/bench_symbols.py on R5 and R2, alternating (round 6)
set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_symbols.py tests/test_r5_list.py tests/test_planted_edges.py -m gpu -x -q --timeout 120 --timeout-method thread -k "symbol or r5 or multibyte" > gpurun_out/ab/sp_tests.log 2>&1
tail -1 gpurun_out/ab/sp_tests.log
for rep in 1 2; do
  DPRF_LIB=$PWD/build/ab/libdprf_sp0.so timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5,pdf_r2,odt > gpurun_out/ab/sp_old_$rep.jsonl 2>/dev/null
  timeout -k 5 200 python tools/bench_symbols.py --formats pdf_r5,pdf_r2,odt > gpurun_out/ab/sp_new_$rep.jsonl 2>/dev/null
done

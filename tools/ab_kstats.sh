#!/bin/bash
# Per-kernel durations of several library builds for one workload: parity tests of that family under each,
# then one rocprofv3 --kernel-trace --stats pass of bench.py per build.
# Usage: tools/ab_kstats.sh <workload> <pytest -k expr> <variant>...   (variant "base" = in-tree)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
W=$1; K=$2; shift 2
for V in "$@"; do
  if [ "$V" = "base" ]; then L=$R/dprf_amd/libdprf.so; else L=$R/build/ab/libdprf_$V.so; fi
  export DPRF_LIB=$L
  timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py tests/test_docs.py -m gpu -x -q --timeout 60 --timeout-method thread -k "$K" > $R/gpurun_out/abk_${V}_tests.log 2>&1
  O=$R/gpurun_out/abk_${V}
  (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o kt --output-format csv -- python3 $R/bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 --warmup 1 > $O.json)
  echo "== $V"
  python3 -c "import json; d=json.load(open('$O.json')); print('value', d['value'])"
  find $O -name "*kernel_stats.csv" -exec cat {} \;
done

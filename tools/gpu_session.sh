#!/bin/bash
# One GPU-box session (gpurun): the GPU test suite, the default bench line, rocprof of every workload, then
# optional A/B library variants.  Every step has its own time limit; the script stops at the first failure.
# Usage (on the box, from the repo root): tools/gpu_session.sh <tag> [ab-workload ab-variants...]
set -e
TAG=${1:?tag}; shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -30 gpurun_out/gputests_$TAG.log; exit 1; }
tail -3 gpurun_out/gputests_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
echo "== bench $(date +%T)"
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['roofline']['frac'], {k: round(v['value']/1e6,3) for k, v in d['per_format'].items()})"
if [ -z "$NO_PROFILE" ]; then
  echo "== profile $(date +%T)"
  bash tools/profile_all.sh $TAG
fi
if [ $# -gt 0 ]; then
  W=$1; shift
  echo "== A/B $W $(date +%T)"
  for V in "$@"; do
    if [ "$V" = "base" ]; then L=$R/dprf_amd/libdprf.so; else L=$R/build/ab/libdprf_$V.so; fi
    for rep in 1 2; do
      DPRF_LIB=$L timeout -k 5 150 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 2 | python -c "import json,sys; d=json.load(sys.stdin); print('$V', d['value'], d['roofline']['frac'])"
    done
  done
fi
echo "== done $(date +%T)"

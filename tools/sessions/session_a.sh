#!/bin/bash
# GPU session A (round 4): GPU tests, smoke, one default bench line.  Usage on the box: tools/session_a.sh <tag>
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -40 gpurun_out/gputests_$TAG.log; exit 1; }
tail -2 gpurun_out/gputests_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(len(open('gpurun_out/bench_$TAG.json').read()), 'bytes'); print(json.dumps(d['summary']))"
echo "== done $(date +%T)"

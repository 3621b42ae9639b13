#!/bin/bash
# round 5 session C: the idregs-default build -- GPU tests, smoke, the chain-latency probe of the shipped header, and
# the default bench line (new fractions, every format's CPU process model)
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
chk() { local rc=$1; if [ $rc -ge 124 ]; then echo "STOP rc=$rc" | tee -a $O/summary.txt; exit $rc; fi; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gputests.log 2>&1; rc=$?
echo "gpu tests rc=$rc $(tail -n 1 $O/gputests.log)" | tee -a $O/summary.txt; chk $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc $(tail -n 1 $O/smoke.log)" | tee -a $O/summary.txt; chk $rc
timeout -k 10 180 build/probe/probe_default time 4000 > $O/latency_default.jsonl 2>&1; rc=$?
echo "latency rc=$rc" | tee -a $O/summary.txt; chk $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?
echo "bench rc=$rc" | tee -a $O/summary.txt; chk $rc
python -c "import json; d=json.load(open('$O/bench.json')); print(json.dumps(d['summary']))" | tee -a $O/summary.txt

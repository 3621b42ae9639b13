#!/bin/bash
# A/B of the product's early-stop rounds vs full verification per format (bench.py --stop-on-first).
set -e
B="python bench.py --no-side --cpu-seconds 0 --steps 3"
for W in ${@:-pdf_r2 pdf_r34 pdf_r5 odt}; do
 timeout -k 10 120 $B --workload $W | python -c "import json,sys; d=json.load(sys.stdin); print('$W full', d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['candidates_per_launch'])"
 timeout -k 10 120 $B --workload $W --stop-on-first | python -c "import json,sys; d=json.load(sys.stdin); print('$W stop', d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['candidates_per_launch'])"
done

set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1
for w in pdf_r34 pdf_r2; do timeout -k 5 100 python bench.py --workload $w --no-side --cpu-seconds 0 --steps 3 | python -c "import json,sys; d=json.load(sys.stdin); print('$w', d['value'], d['roofline']['frac'])"; done

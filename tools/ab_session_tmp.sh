set -e
bash tools/gpu_session.sh r03b
echo "== n2 library-mode rehearsal $(date +%T)"
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 200 python bench.py --gpus 2 --no-side --cpu-seconds 0 --no-cluster > gpurun_out/bench_lanes2_r03b.json 2> gpurun_out/bench_lanes2_r03b.err
python -c "import json; d=json.load(open('gpurun_out/bench_lanes2_r03b.json')); print(d['value'], d.get('device_balance',{}).get('last_over_mean'))"
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --workload pdf_r6 --no-side --cpu-seconds 0 --no-cluster --steps 2 > gpurun_out/bench_lanes2_r6_r03b.json 2>> gpurun_out/bench_lanes2_r03b.err
python -c "import json; d=json.load(open('gpurun_out/bench_lanes2_r6_r03b.json')); print(d['value'], d.get('device_balance',{}).get('last_over_mean'))"

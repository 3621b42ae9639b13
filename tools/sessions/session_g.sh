#!/bin/bash
# GPU session G (round 4): the N>1 bench paths on the one-GPU box -- the library's multi-device path (two device
# lanes on device 0) and the driver's torchrun path (two ranks on device 0, gloo for the exchanges).
set -e
TAG=${1:?tag}
mkdir -p gpurun_out
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 400 python bench.py --gpus 2 --no-side --cpu-seconds 0 --steps 3 > gpurun_out/bench_lanes2_$TAG.json 2> gpurun_out/bench_lanes2_$TAG.err || { tail -20 gpurun_out/bench_lanes2_$TAG.err; exit 1; }
DPRF_BENCH_SAME_DEVICE=1 DPRF_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 --side-steps 2 > gpurun_out/bench_n2_rehearsal_$TAG.json 2> gpurun_out/bench_n2_rehearsal_$TAG.err || { tail -20 gpurun_out/bench_n2_rehearsal_$TAG.err; exit 1; }
python -c "
import json
for f in ('bench_lanes2_$TAG.json', 'bench_n2_rehearsal_$TAG.json'):
    d = json.loads(open('gpurun_out/' + f).read().strip().splitlines()[-1])
    print(f, d['n_gpus'], d['value'], json.dumps(d.get('summary', {}).get('workloads', {}))[:600])
"
echo "== done $(date +%T)"

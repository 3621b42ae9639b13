#!/bin/bash
# round 5 session F: the N>1 paths on the one-GPU box on the round-5 build -- the library's
# multi-device path (two device lanes on device 0, with device_balance) and the driver's torchrun path (two ranks on
# device 0, gloo for the exchanges RCCL refuses on one GPU); every per-format leg runs in the torchrun rehearsal.
set -o pipefail
TAG=${1:?tag}
mkdir -p gpurun_out
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --no-side --cpu-seconds 0 --steps 3 > gpurun_out/bench_lanes2_$TAG.json 2> gpurun_out/bench_lanes2_$TAG.err || { tail -20 gpurun_out/bench_lanes2_$TAG.err; exit 1; }
DPRF_BENCH_SAME_DEVICE=1 DPRF_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 --no-cluster > gpurun_out/bench_n2_rehearsal_$TAG.json 2> gpurun_out/bench_n2_rehearsal_$TAG.err || { tail -20 gpurun_out/bench_n2_rehearsal_$TAG.err; exit 1; }
python -c "
import json
for f in ('bench_lanes2_$TAG.json', 'bench_n2_rehearsal_$TAG.json'):
    d = json.loads(open('gpurun_out/' + f).read().strip().splitlines()[-1])
    print(f, d['value'], d['n_gpus'], {k: round(v['value'] / 1e6, 3) for k, v in d.get('per_format', {}).items()}, d.get('device_balance', {}).get('last_over_mean'))
"

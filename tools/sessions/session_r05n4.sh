#!/bin/bash
# round 5: N = 4 rehearsals on the one-GPU box (final build): the library's four device lanes on device 0 with
# device_balance, and torchrun with four ranks on device 0 (gloo for the exchanges RCCL refuses on one GPU; the
# headline leg only -- four ranks share the one GPU, so every leg takes four times as long).  A heartbeat file keeps
# the box's silence watchdog informed while the ranks run.
set -o pipefail
O=gpurun_out/r05n4
mkdir -p $O
(while sleep 45; do date >> $O/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 4 --no-side --cpu-seconds 0 --steps 3 > $O/bench_lanes4.json 2> $O/bench_lanes4.err || exit 1
DPRF_BENCH_SAME_DEVICE=1 DPRF_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 4 --steps 2 --warmup 1 --cpu-seconds 0 --no-side --no-cluster > $O/bench_n4_rehearsal.json 2> $O/bench_n4_rehearsal.err || exit 1
python -c "
import json
for f in ('bench_lanes4.json', 'bench_n4_rehearsal.json'):
    d = json.loads(open('$O/' + f).read().strip().splitlines()[-1])
    b = d.get('device_balance') or {}
    print(f, d['value'], d['n_gpus'], {k: v for k, v in b.items() if k != 'devices'})
"

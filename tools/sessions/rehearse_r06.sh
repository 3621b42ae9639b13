#!/bin/bash
# The N>1 paths on the one-GPU box, on the final round-6 build (run once, VERDICT r5 Next #7): two and four library
# device lanes on device 0, the driver's torchrun path with two ranks on device 0 (gloo), and the RCCL branch with one
# rank.  The r06d profiles are installed in profiles/ so the lines read counters of the same build.
set -e
T=${1:-r06d}
mkdir -p gpurun_out
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --no-side --cpu-seconds 0 --steps 3 > gpurun_out/bench_lanes2_$T.json 2> gpurun_out/bench_lanes2_$T.err
DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 4 --no-side --cpu-seconds 0 --steps 3 > gpurun_out/bench_lanes4_$T.json 2> gpurun_out/bench_lanes4_$T.err
DPRF_BENCH_SAME_DEVICE=1 DPRF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_n2_rehearsal_$T.json 2> gpurun_out/bench_n2_rehearsal_$T.err
DPRF_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-side > gpurun_out/bench_rccl1_rehearsal_$T.json 2> gpurun_out/bench_rccl1_rehearsal_$T.err
python -c "import json; [print(f, json.loads(open('gpurun_out/'+f).read().strip().splitlines()[-1])['value']) for f in ('bench_lanes2_$T.json', 'bench_lanes4_$T.json', 'bench_n2_rehearsal_$T.json', 'bench_rccl1_rehearsal_$T.json')]"

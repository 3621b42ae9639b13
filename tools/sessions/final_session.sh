#!/bin/bash
# The end-of-round GPU session (gpurun): GPU tests, smoke, rocprof of every workload on THIS build, the profiles
# installed into profiles/ (box-local) so that the bench line that follows reads counters of the same build
# ("stale": false), then the bench line.  Everything to keep is copied under gpurun_out/.
# Usage (on the box, from the repo root): tools/sessions/final_session.sh <tag>
set -e
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
echo "== tests $(date +%T)"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -30 gpurun_out/gputests_$TAG.log; exit 1; }
tail -1 gpurun_out/gputests_$TAG.log
echo "== smoke $(date +%T)"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
echo "== profile $(date +%T)"
bash tools/profile_all.sh $TAG
for W in odt office odt_e pdf_r34 pdf_r3 pdf_r3_40 pdf_r6 pdf_r2 pdf_r5; do
  cp gpurun_out/summary_${W}_$TAG.json profiles/prof_${W}_$TAG.json
  cp gpurun_out/summary_${W}_${TAG}_kernel_stats.csv profiles/prof_${W}_${TAG}_kernel_stats.csv
done
python3 tools/pmc_traffic.py $TAG > /dev/null
cp profiles/pmc_traffic.json profiles/pmc_valu.json gpurun_out/
echo "== bench $(date +%T)"
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); r=d['roofline']; print(d['value'], r['frac'], r['bound'], r['rocprof']['stale'], r['traffic_source']['stale'], {k: (round(v['value']/1e6,3), v.get('rocprof',{}).get('stale')) for k, v in d['per_format'].items()})"
if [ -n "$REHEARSE" ]; then
  # the N>1 paths on the one-GPU box, same build: the library's multi-device path (two device lanes on device 0) and
  # the driver's torchrun path (two ranks on device 0, gloo for the exchanges RCCL refuses on one GPU)
  echo "== rehearsals $(date +%T)"
  DPRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --no-side --cpu-seconds 0 --steps 3 > gpurun_out/bench_lanes2_$TAG.json 2> gpurun_out/bench_lanes2_$TAG.err || { tail -20 gpurun_out/bench_lanes2_$TAG.err; exit 1; }
  DPRF_BENCH_SAME_DEVICE=1 DPRF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_n2_rehearsal_$TAG.json 2> gpurun_out/bench_n2_rehearsal_$TAG.err || { tail -20 gpurun_out/bench_n2_rehearsal_$TAG.err; exit 1; }
  # and the RCCL branch the driver's N>1 runs take (one rank, so RCCL accepts it): process group, barriers and the
  # MIN / MAX all-reduces on device tensors
  DPRF_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-side > gpurun_out/bench_rccl1_rehearsal_$TAG.json 2> gpurun_out/bench_rccl1_rehearsal_$TAG.err || { tail -20 gpurun_out/bench_rccl1_rehearsal_$TAG.err; exit 1; }
  python -c "import json; [print(f, json.loads(open('gpurun_out/'+f).read().strip().splitlines()[-1])['value']) for f in ('bench_lanes2_$TAG.json', 'bench_n2_rehearsal_$TAG.json', 'bench_rccl1_rehearsal_$TAG.json')]"
fi
echo "== done $(date +%T)"

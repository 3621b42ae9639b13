#!/bin/bash
# Final-build sessions of round 4, split so each call stays well under gpurun's limit:
#   tools/session_f.sh <tag> 1   GPU tests + smoke + rocprof of odt office odt_e pdf_r34 pdf_r3
#   tools/session_f.sh <tag> 2   rocprof of pdf_r3_40 pdf_r6 pdf_r2 pdf_r5, then pmc_traffic + the bench line (reads the
#                                 summaries of part 1, copied into profiles/ on the CPU side before part 2 is sent)
set -e
TAG=${1:?tag}; PART=${2:?part}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
if [ "$PART" = 1 ]; then
  echo "== tests $(date +%T)"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_$TAG.log 2>&1 || { tail -30 gpurun_out/gputests_$TAG.log; exit 1; }
  tail -1 gpurun_out/gputests_$TAG.log
  echo "== smoke $(date +%T)"
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { cat gpurun_out/smoke_$TAG.log; exit 1; }
  WL="odt office odt_e pdf_r34 pdf_r3"
else
  WL="pdf_r3_40 pdf_r6 pdf_r2 pdf_r5"
fi
echo "== profile $WL $(date +%T)"
bash tools/profile_all.sh $TAG $WL
for W in $WL; do
  cp gpurun_out/summary_${W}_$TAG.json profiles/prof_${W}_$TAG.json
  cp gpurun_out/summary_${W}_${TAG}_kernel_stats.csv profiles/prof_${W}_${TAG}_kernel_stats.csv
done
if [ "$PART" = 2 ]; then
  python3 tools/pmc_traffic.py $TAG > /dev/null
  cp profiles/pmc_traffic.json profiles/pmc_valu.json gpurun_out/
  echo "== bench $(date +%T)"
  timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(json.dumps(d['summary'])); r=d['roofline']; print(r['frac'], r['rocprof'].get('stale'), r['traffic_source'].get('stale'), {k: (v.get('rocprof') or {}).get('stale') for k, v in d['per_format'].items()})"
fi
echo "== done $(date +%T)"

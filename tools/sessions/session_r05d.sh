#!/bin/bash
# round 5 session D: the first-dispatch write excess of k_pdf_r6.  Alternating PMC runs of the R6
# bench step with the library's queue warm-up off (DPRF_NO_QUEUE_WARMUP=1, the round-4 behaviour) and on; each run
# collects WRITE_SIZE + SQ_WAVES + GRBM_GUI_ACTIVE per dispatch in ONE pass (tools/first_dispatch.py reads them).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05d
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for V in nowarm warm; do
    D=$O/${V}_$rep
    if [ $V = nowarm ]; then export DPRF_NO_QUEUE_WARMUP=1; else unset DPRF_NO_QUEUE_WARMUP; fi
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d $D -o w --output-format csv \
        -- python3 $R/bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 > $D.json 2> $D.err
    rc=$?
    echo "$V $rep rc=$rc" >> $O/summary.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
    python3 $R/tools/first_dispatch.py $D >> $O/first_dispatch.jsonl
  done
done
unset DPRF_NO_QUEUE_WARMUP

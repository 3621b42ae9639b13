#!/bin/bash
# GPU session B (round 4): R2-R4 KSA A/B (parity of each variant, then alternating bench runs), and the WRITE_SIZE
# outlier check (odt_e / pdf_r6 write passes over several dispatches).  Usage on the box: tools/session_b.sh <tag> [variants]
set -e
TAG=${1:?tag}; shift
VARS=${@:-r24_ic4 r24_d16merge r24_ic4_d16merge r24_split_add r24_split_add_ic4 r24_split_add_ic4_d16merge}
mkdir -p gpurun_out
for V in $VARS; do
  echo "== parity $V $(date +%T)"
  DPRF_LIB=$PWD/build/ab/libdprf_$V.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 100 --timeout-method thread -k "hitsets_match or verdict_tables_match or truncates" > gpurun_out/ab_${V}_$TAG.log 2>&1 || { tail -20 gpurun_out/ab_${V}_$TAG.log; exit 1; }
  tail -1 gpurun_out/ab_${V}_$TAG.log
done
for rep in 1 2 3; do
  for V in base $VARS; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    for W in pdf_r34 pdf_r2; do
      DPRF_LIB=$L timeout -k 5 120 python bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$rep $V $W', round(d['value']/1e6,2), round(d['roofline']['kernel_avg_ms'],3))"
    done
  done
done
echo "== write outliers $(date +%T)"
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for W in odt_e pdf_r6; do
  timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/wr_${W}_$TAG -o wr --output-format csv -- python3 $R/bench.py --workload $W --no-side --cpu-seconds 0 --steps 3 --warmup 1 > /dev/null
done
cd $R
python3 - <<'PY'
import csv, glob
for w in ("odt_e", "pdf_r6"):
    for f in glob.glob("gpurun_out/wr_%s_*/**/*counter_collection.csv" % w, recursive=True):
        print(w, [(r["Dispatch_Id"], round(float(r["Counter_Value"]))) for r in csv.DictReader(open(f)) if "k_" in r["Kernel_Name"] and ("kdf" in r["Kernel_Name"] or "r6" in r["Kernel_Name"])])
PY
echo "== done $(date +%T)"

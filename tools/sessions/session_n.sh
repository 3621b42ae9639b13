#!/bin/bash
# GPU session N (round 4): PDF R6 bank-placed claims (R6_BANK_PLACE: the first two queued slots of each bank residue
# on lanes b / 32 + b) -- parity, PMC bank conflicts, alternating bench runs against the product build
set -e
mkdir -p gpurun_out
DPRF_LIB=$PWD/build/ab/libdprf_r6_place.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py -m gpu -x -q --timeout 200 --timeout-method thread -k "r6 or R6" 2>&1 | tail -1
for V in base r6_place; do
  if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
  DPRF_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/n_lds_$V -o lds --output-format csv -- python3 bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 1 --warmup 0 --batch 8388608 > /dev/null
  python3 - gpurun_out/n_lds_$V $V <<'PY'
import csv, glob, sys, collections
f = [p for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)][0]
tot = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "k_pdf_r6" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
cyc = tot["GRBM_GUI_ACTIVE"] / 8 * 256
print(sys.argv[2], "conflict/CU-cycles %.4f" % (tot["SQ_LDS_BANK_CONFLICT"] / cyc), "conflict/LDS-active %.4f" % (tot["SQ_LDS_BANK_CONFLICT"] / tot["SQ_LDS_IDX_ACTIVE"]), "wait_any %.3f" % (tot["SQ_WAIT_ANY"] / tot["SQ_WAVE_CYCLES"]))
PY
done
for rep in 1 2 3; do
  for V in base r6_place; do
    if [ "$V" = "base" ]; then L=$PWD/dprf_amd/libdprf.so; else L=$PWD/build/ab/libdprf_$V.so; fi
    DPRF_LIB=$L timeout -k 5 150 python bench.py --workload pdf_r6 --no-side --cpu-seconds 0 --steps 2 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print('$rep $V', round(d['value']/1e6,4), round(d['roofline']['kernel_avg_ms'],1))"
  done
done
echo "== done $(date +%T)"

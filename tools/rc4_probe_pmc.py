#!/usr/bin/env python3
"""Per-dispatch SQ counters of `rc4_ksa_probe time` under rocprofv3 (tools/sessions/session_r05k.sh): for each number of
one-wave workgroups per CU, where a chain's wave-cycles go -- parked on s_waitcnt (SQ_WAIT_ANY: the LDS round trips),
ready but not issued (SQ_WAIT_INST_ANY: another wave holds the issue port) -- and the VALU / LDS instructions issued.
Usage: tools/rc4_probe_pmc.py gpurun_out/r05k/pmc"""
import collections
import csv
import glob
import json
import sys

f = glob.glob(sys.argv[1] + "/**/*_counter_collection.csv", recursive=True)[0]
per = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for r in csv.DictReader(open(f)):
    if not r["Kernel_Name"].startswith("void k_time"):
        continue
    d = int(r["Dispatch_Id"])
    per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    meta[d] = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
rows = collections.defaultdict(list)
for d, c in per.items():
    k, grid, ns = meta[d]
    wpc = grid // 64 // 256
    wc = c["SQ_WAVE_CYCLES"]
    rows[(k, wpc)].append({"dispatch": d, "ms": ns / 1e6, "wait_any": c["SQ_WAIT_ANY"] / wc, "wait_inst_any": c["SQ_WAIT_INST_ANY"] / wc,
                           "valu_insts_per_wave_cycle": c["SQ_INSTS_VALU"] / wc, "lds_insts_per_wave_cycle": c["SQ_INSTS_LDS"] / wc,
                           "valu_busy": c["SQ_ACTIVE_INST_VALU"] * 4 / 1024 / (c["GRBM_GUI_ACTIVE"] / 8),
                           "clock_GHz": c["GRBM_GUI_ACTIVE"] / 8 / ns})
for (k, wpc), rs in sorted(rows.items()):
    r = max(rs, key=lambda x: x["dispatch"])    # the last dispatch of that shape: a timed one, after the warm-up
    print(json.dumps({"kernel": k, "waves_per_cu": wpc, **{a: round(b, 4) for a, b in r.items()}}))

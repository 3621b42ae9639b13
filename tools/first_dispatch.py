#!/usr/bin/env python3
"""Per-dispatch WRITE_SIZE / SQ_WAVES of one rocprofv3 --pmc run (round 5, VERDICT r4 "next" #6: who writes the
~177 MB extra in the FIRST k_pdf_r6 dispatch of some processes).

Each run is `rocprofv3 --pmc WRITE_SIZE SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -- python3 bench.py --workload pdf_r6
--steps 1 --warmup 0` (tools/sessions/session_r05d.sh).  A context save of the resident waves (CWSR: the scheduler preempting
the queue) writes every wave's VGPRs + SGPRs and every CU's LDS; a restored wave is launched again, so SQ_WAVES of
that dispatch exceeds its grid.  Printed per dispatch: candidates (from the trace duration share), WRITE bytes per
candidate, SQ_WAVES, and the expected size of a whole-chip context save from the kernel's resources.

Usage: tools/first_dispatch.py <run dir> [<run dir> ...]   ->  one JSON line per run
"""
import collections
import csv
import glob
import json
import os
import sys


def run(d):
    f = glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True)
    if not f:
        return {"dir": d, "error": "no counter csv"}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0]
        if k.startswith("__amd"):
            continue
        i = int(r["Dispatch_Id"])
        per[i][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[i] = {"kernel": k, "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                   "grid": int(r.get("Grid_Size", 0) or 0), "wg": int(r.get("Workgroup_Size", 0) or 0),
                   "lds": int(r.get("LDS_Block_Size", r.get("Lds_Size", 0)) or 0),
                   "vgpr": int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0),
                   "agpr": int(r.get("Accum_VGPR_Count", 0) or 0), "sgpr": int(r.get("SGPR_Count", 0) or 0)}
    ids = sorted(i for i in per if meta[i]["kernel"].startswith("void k_pdf_r6") or "k_pdf_r6" in meta[i]["kernel"])
    out = []
    for i in ids:
        m = meta[i]
        waves = m["grid"] // 64 if m["grid"] else None
        out.append({"dispatch": i, "ms": m["ns"] / 1e6, "write_KiB": per[i].get("WRITE_SIZE"),
                    "sq_waves": per[i].get("SQ_WAVES"), "grid_waves": waves, "vgpr": m["vgpr"], "agpr": m["agpr"],
                    "sgpr": m["sgpr"], "lds": m["lds"]})
    tot_ns = sum(o["ms"] for o in out) or 1
    return {"dir": d, "dispatches": out}


if __name__ == "__main__":
    for d in sys.argv[1:]:
        print(json.dumps(run(d)))

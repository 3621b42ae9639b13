#!/usr/bin/env python3
"""Collect the dominant kernel's PMC figures from the profile summaries (tools/prof_summary.py output):
  profiles/pmc_traffic.json  HBM bytes per candidate and per profiled launch (FETCH_SIZE + WRITE_SIZE) ->
                             bench.py roofline.traffic (per candidate x bench's own candidates per launch)
  profiles/pmc_valu.json     VALUBusy, VALUUtilization, LDS busy, effective clock -> bench.py roofline.valu_busy

FETCH_SIZE / WRITE_SIZE come from separate rocprofv3 --pmc passes (they cannot share one on gfx950) and are
in KiB.  MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of WIDE streaming reads (16 B/lane); none of these kernels
streams its inputs (document constants are kernel arguments / a few KiB of tables), so no correction is
applied.  Usage: tools/pmc_traffic.py r02 [r02b ...] (for each workload the last tag that has a profile wins)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CUS, XCDS, SIMDS = 256, 8, 1024
PMC_STEPS = 2          # tools/profile_gpu.sh counts two steps of bench.py per PMC pass (prof_summary.py)
DOM = {"odt": "k_odt_kdf", "odt_e": "k_odt_kdf", "office": "k_office_kdf", "pdf_r34": "k_pdf_r24",
       "pdf_r3": "k_pdf_r24", "pdf_r3_40": "k_pdf_r24", "pdf_r2": "k_pdf_r24", "pdf_r5": "k_pdf_r5",
       "pdf_r6": "k_pdf_r6"}
tags = sys.argv[1:] or ["r02"]
traffic, valu = {}, {}
for w, kname in DOM.items():
    f = None
    for tag in tags:
        cand = os.path.join(HERE, "profiles", "prof_%s_%s.json" % (w, tag))
        if os.path.exists(cand):
            f = cand
    if f is None:
        continue
    d = json.load(open(f))
    build = d.get("build")
    for k, v in d.get("counters", {}).items():
        if kname not in k:
            continue
        pd = v["per_dispatch"]
        src = os.path.relpath(f, HERE)
        if v.get("hbm_bytes_per_dispatch") is not None:
            traffic[w] = {"kernel": k, "bytes_per_launch": v.get("hbm_bytes_per_dispatch"),
                          "bytes_per_candidate": v.get("hbm_bytes_per_candidate"),
                          "fetch_bytes": pd.get("FETCH_SIZE", 0) * 1024, "write_bytes": pd.get("WRITE_SIZE", 0) * 1024,
                          "source": src, "build": build}
        if v.get("valu_busy") is not None:
            # the issue line (round 6): wave-instructions per candidate lane over the counted steps'
            # dispatches (bench.py --steps 2: 2 x batch candidates), and SIMD cycles per wave-instruction within the
            # SQ pass (GRBM_GUI_ACTIVE / XCDs = the dispatch's cycles on every CU)
            batch = ((d.get("bench_under_profiler") or {}).get("config") or {}).get("batch_per_gpu")
            tot = v.get("per_run_total", {})
            sq = v.get("passes", {}).get("sq", {})
            ipc = tot["SQ_INSTS_VALU"] * 64 / (batch * PMC_STEPS) if batch and tot.get("SQ_INSTS_VALU") else None
            cpi = (sq["GRBM_GUI_ACTIVE"] / XCDS * SIMDS / sq["SQ_INSTS_VALU"]
                   if sq.get("GRBM_GUI_ACTIVE") and sq.get("SQ_INSTS_VALU") else None)
            valu[w] = {"kernel": k, "valu_busy": v.get("valu_busy"), "valu_utilization": v.get("valu_utilization"),
                       "valu_instr_per_candidate": ipc, "cycles_per_valu_instr": cpi,
                       "lds_busy": v.get("lds_busy"), "lds_util": v.get("lds_util"),
                       "effective_clock_GHz": v.get("effective_clock_GHz"),
                       "valu_active_per_wave_cycle": v.get("valu_active_per_wave_cycle"),
                       "wait_any_frac": v.get("wait_any_frac"), "wait_inst_any_frac": v.get("wait_inst_any_frac"),
                       "SQ_LDS_BANK_CONFLICT_per_launch": pd.get("SQ_LDS_BANK_CONFLICT"),
                       # bank-conflict cycles (summed over the CUs) per CU cycle of the dispatch
                       "lds_bank_conflict_frac": (pd["SQ_LDS_BANK_CONFLICT"] / (CUS * pd["GRBM_GUI_ACTIVE"] / XCDS)
                                                  if pd.get("SQ_LDS_BANK_CONFLICT") is not None and pd.get("GRBM_GUI_ACTIVE")
                                                  else None),
                       "source": src, "build": build}
for name, obj in (("pmc_traffic.json", traffic), ("pmc_valu.json", valu)):
    json.dump(obj, open(os.path.join(HERE, "profiles", name), "w"), indent=1)
print(json.dumps({"traffic": traffic, "valu": valu}, indent=1))

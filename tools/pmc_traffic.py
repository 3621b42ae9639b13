#!/usr/bin/env python3
"""Collect the dominant kernel's HBM bytes per launch from the profile summaries (tools/prof_summary.py
output) into profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.

FETCH_SIZE / WRITE_SIZE come from separate rocprofv3 --pmc passes (they cannot share one on gfx950) and are
in KiB.  MI355X_MICROARCH.md: FETCH_SIZE reads 1/2 of WIDE streaming reads (16 B/lane); none of these kernels
streams its inputs (document constants are kernel arguments / a few KiB of tables), so no correction is
applied.  Usage: tools/pmc_traffic.py r01 [r01b ...] (for each workload the last tag that has a profile wins)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOM = {"odt": "k_odt_kdf", "odt_e": "k_odt_kdf", "office": "k_office_kdf", "pdf_r34": "k_pdf_r24",
       "pdf_r2": "k_pdf_r24", "pdf_r5": "k_pdf_r5", "pdf_r6": "k_pdf_r6"}
tags = sys.argv[1:] or ["r01"]
out = {}
for w, kname in DOM.items():
    f = None
    for tag in tags:
        cand = os.path.join(HERE, "profiles", "prof_%s_%s.json" % (w, tag))
        if os.path.exists(cand):
            f = cand
    if f is None:
        continue
    d = json.load(open(f))
    for k, v in d.get("counters", {}).items():
        if kname in k:
            pd = v["per_dispatch"]
            out[w] = {"kernel": k, "bytes_per_launch": v.get("hbm_bytes_per_dispatch"),
                      "fetch_bytes": pd.get("FETCH_SIZE", 0) * 1024, "write_bytes": pd.get("WRITE_SIZE", 0) * 1024,
                      "source": os.path.relpath(f, HERE)}
json.dump(out, open(os.path.join(HERE, "profiles", "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(out, indent=1))

#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh run into profiles/<name>.json + the kernel_stats csv.
Usage: tools/prof_summary.py gpurun_out/prof_odt_r02 profiles/prof_odt_r02

Counters are kept per --pmc pass (each pass is its own run of the program), averaged over the dispatches of
each kernel (FETCH_SIZE / WRITE_SIZE: the median dispatch, see below), and the derived metrics are computed within
one pass:
  valu_busy        = SQ_ACTIVE_INST_VALU * 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs)   (ROCm's VALUBusy formula,
                     derived_counters.xml; GRBM_GUI_ACTIVE is summed over the 8 XCDs on gfx950,
                     MI355X_MICROARCH.md)
  valu_utilization = SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU * 64)           (ROCm's VALUUtilization)
  lds_busy         = SQ_ACTIVE_INST_LDS * 4 / SIMDs / (GRBM_GUI_ACTIVE / XCDs)    (same form, LDS instructions)
  lds_util         = SQ_LDS_IDX_ACTIVE / CUs / (GRBM_GUI_ACTIVE / XCDs)            (ROCm's LdsUtil: LDS-array cycles)
  effective_clock  = GRBM_GUI_ACTIVE / XCDs / kernel duration
HBM bytes are also given per candidate (each PMC pass runs bench.py --steps 1 --warmup 0, i.e. exactly one
batch of candidates, whatever launch sizes the adaptive chunking chose), so bench.py can scale them to its own
launch size; and the kernel-trace pass reports the mean duration of the dominant kernel over the TIMED
dispatches only (the last steps x launches-per-step), the figure bench.py's roofline.kernel_avg_ms measures.
"""
import collections
import csv
import json
import os
import shutil
import sys

SIMDS, XCDS, CUS = 256 * 4, 8, 256
PASSES = ("fetch", "write", "sq", "lds")
PMC_STEPS = 2          # tools/profile_gpu.sh: --steps 2 --warmup 1 for every --pmc pass (round 5: the counted steps
                       # are the last, at the steady-state launch size -- their dispatches are the last per_step x 2 of
                       # each pass -- and two of them, so one context-saved dispatch still leaves a clean one)


def timed_dispatches(src, bench):
    """Mean duration of the dominant kernel over the timed dispatches of the kernel-trace pass."""
    f = os.path.join(src, "kt", "kt_kernel_trace.csv")
    roof = (bench or {}).get("roofline") or {}
    if not os.path.exists(f) or not roof.get("candidates_per_launch"):
        return None
    rows = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        if not k.startswith("__amd"):
            rows[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    dom = max(rows, key=lambda k: sum(d for _, d in rows[k]))
    per_step = max(1, round(bench["config"]["batch_per_gpu"] / roof["candidates_per_launch"]))
    n = per_step * bench["steps"]
    durs = [d for _, d in sorted(rows[dom])][-n:]
    return {"kernel": dom, "dispatches": len(durs), "avg_ns": sum(durs) / len(durs),
            "all_dispatches": len(rows[dom]), "all_avg_ns": sum(d for _, d in rows[dom]) / len(rows[dom])}


def summarize(src, dst):
    os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
    out = {"source": src}
    kt = os.path.join(src, "kt", "kt_kernel_stats.csv")
    if os.path.exists(kt):
        shutil.copy(kt, dst + "_kernel_stats.csv")
        out["kernel_stats"] = [dict(r) for r in csv.DictReader(open(kt))]
    bench = os.path.join(src, "bench_under_kt.json")
    if os.path.exists(bench):
        try:
            out["bench_under_profiler"] = json.load(open(bench))
        except ValueError:
            pass
    bp = out.get("bench_under_profiler")
    # the library build the profile measured (bench.py config.build = dprf_build_id()): bench.py marks counter
    # fields taken from a different build "stale"
    out["build"] = ((bp or {}).get("config") or {}).get("build")
    t = timed_dispatches(src, bp)
    if t:
        out["timed_kernel"] = t
    batch = ((bp or {}).get("config") or {}).get("batch_per_gpu")
    # kernel -> pass -> counter -> {dispatch: value}
    raw = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(dict)))
    dur = collections.defaultdict(lambda: collections.defaultdict(dict))
    grid = collections.defaultdict(lambda: collections.defaultdict(dict))
    roof = (bp or {}).get("roofline") or {}
    # dispatches of the counted (last) step: the bench's launches per step (kernel-trace pass) x PMC_STEPS
    per_step = (max(1, round(batch / roof["candidates_per_launch"]))
                if batch and roof.get("candidates_per_launch") else None)
    for sub in PASSES:
        f = os.path.join(src, sub, sub + "_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if k.startswith("__amd"):
                continue
            d = r["Dispatch_Id"]
            raw[k][sub][r["Counter_Name"]][d] = raw[k][sub][r["Counter_Name"]].get(d, 0.0) + float(r["Counter_Value"])
            dur[k][sub][d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            grid[k][sub][d] = int(r.get("Grid_Size") or 0)
    summ = {}
    for k, passes_all in raw.items():
        per = {"per_dispatch": {}, "passes": {}}
        # round 5: only the counted step's dispatches (the warm-up step before it runs the first, smaller launches)
        passes = {}
        for sub, ctrs in passes_all.items():
            ids = sorted(dur[k][sub], key=int)
            keep = set(ids[-per_step * PMC_STEPS:] if per_step else ids)
            passes[sub] = {name: {d: v for d, v in vals.items() if d in keep} for name, vals in ctrs.items()}
            dur[k][sub] = {d: t for d, t in dur[k][sub].items() if d in keep}
        # context saves (round 5): a dispatch whose waves were saved and restored counts them twice in
        # SQ_WAVES, and its HBM bytes include the save of every resident wave's registers and the CUs' LDS (~140-180 MB)
        saves = {}
        for sub, ctrs in passes.items():
            for d, w in ctrs.get("SQ_WAVES", {}).items():
                g = grid[k][sub].get(d, 0)
                if g and w > 1.05 * ((g + 63) // 64):
                    saves.setdefault(sub, []).append(d)
        for sub, ctrs in passes.items():
            avg = {name: sum(v.values()) / len(v) for name, v in ctrs.items()}
            # HBM byte counters (round 4): every dispatch's value is recorded, and per_dispatch holds the MEDIAN dispatch
            # (round 3's r03i profiles had one dispatch at 2-3x the others -- odt_e 269,946 vs 131,072 KiB, R6 260,698 vs
            # 83,2xx KiB -- which a re-check over 16 + 10 dispatches did not reproduce: profiles/write_size_recheck_r04b.json).
            # Bytes per CANDIDATE: below (per dispatch, by duration share -- R6's launches differ in size within a run, 2^22
            # until the rate is measured, then ~2^25, where a median dispatch says nothing per candidate).
            for name in ("FETCH_SIZE", "WRITE_SIZE"):
                if name in ctrs:
                    vals = [ctrs[name][d] for d in sorted(ctrs[name], key=int) if d not in saves.get(sub, [])] or \
                        [ctrs[name][d] for d in sorted(ctrs[name], key=int)]
                    med = sorted(vals)[len(vals) // 2] if len(vals) % 2 else sum(sorted(vals)[len(vals) // 2 - 1:len(vals) // 2 + 1]) / 2
                    avg[name] = med
                    per.setdefault("hbm_dispatch_values", {})[name] = vals
                    out_d = [i for i, v in enumerate(vals) if med > 0 and v > 1.2 * med]
                    if out_d:
                        per.setdefault("hbm_outlier_dispatches", {})[name] = out_d
            ns = sum(dur[k][sub].values()) / max(1, len(dur[k][sub]))
            per["passes"][sub] = dict(avg, kernel_ns=ns, dispatches=len(dur[k][sub]))
            per.setdefault("per_run_total", {}).update({name: sum(v.values()) for name, v in ctrs.items()})
            per["per_dispatch"].update(avg)
            g = avg.get("GRBM_GUI_ACTIVE")
            if g:
                cyc = g / XCDS
                per.setdefault("effective_clock_GHz", cyc / ns if ns else None)
                if "SQ_ACTIVE_INST_VALU" in avg:
                    per["valu_busy"] = avg["SQ_ACTIVE_INST_VALU"] * 4 / SIMDS / cyc
                if "SQ_ACTIVE_INST_LDS" in avg:
                    per["lds_busy"] = avg["SQ_ACTIVE_INST_LDS"] * 4 / SIMDS / cyc
                if "SQ_LDS_IDX_ACTIVE" in avg:
                    # ROCm's LdsUtil: LDS-array cycles of indexed operations over the CUs' cycles (the fraction of
                    # the LDS pipeline in use; SQ_ACTIVE_INST_LDS above counts instruction issue on the SIMDs)
                    per["lds_util"] = avg["SQ_LDS_IDX_ACTIVE"] / (CUS * cyc)
                if "SQ_LDS_BANK_CONFLICT" in avg:
                    per["lds_bank_conflict_frac"] = avg["SQ_LDS_BANK_CONFLICT"] / (CUS * cyc)
            if avg.get("SQ_THREAD_CYCLES_VALU") and avg.get("SQ_ACTIVE_INST_VALU"):
                per["valu_utilization"] = avg["SQ_THREAD_CYCLES_VALU"] / (avg["SQ_ACTIVE_INST_VALU"] * 64)
            if avg.get("SQ_ACTIVE_INST_VALU") and avg.get("SQ_WAVE_CYCLES"):
                per["valu_active_per_wave_cycle"] = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
        pd = per["per_dispatch"]
        # where the waves' time goes (MI355X_MICROARCH.md PMC table: WAIT_ANY = parked on s_waitcnt / barrier,
        # WAIT_INST_ANY = an instruction ready but not issued; both in the units of SQ_WAVE_CYCLES, which comes from
        # another pass of the same workload: ratios of two runs)
        if pd.get("SQ_WAVE_CYCLES"):
            if "SQ_WAIT_ANY" in pd:
                per["wait_any_frac"] = pd["SQ_WAIT_ANY"] / pd["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_INST_ANY" in pd:
                per["wait_inst_any_frac"] = pd["SQ_WAIT_INST_ANY"] / pd["SQ_WAVE_CYCLES"]
        if saves:
            per["context_saves"] = {sub: [{"dispatch": d, "sq_waves": passes[sub]["SQ_WAVES"][d],
                                           "grid_waves": (grid[k][sub][d] + 63) // 64,
                                           "bytes": {n: passes[sub][n][d] * 1024 for n in ("FETCH_SIZE", "WRITE_SIZE")
                                                     if d in passes[sub].get(n, {})}} for d in ds]
                                    for sub, ds in saves.items()}
        if "FETCH_SIZE" in pd or "WRITE_SIZE" in pd:
            # rocprofv3 FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reads 1/2 of wide streaming
            # reads (MI355X_MICROARCH.md HBM section) -- these kernels have no streaming reads, no correction.
            per["hbm_bytes_per_dispatch"] = (pd.get("FETCH_SIZE", 0) + pd.get("WRITE_SIZE", 0)) * 1024
            if batch:
                tot = per["per_run_total"]
                per["pmc_candidates"] = batch * PMC_STEPS
                per["hbm_bytes_per_candidate_run_total"] = (tot.get("FETCH_SIZE", 0) + tot.get("WRITE_SIZE", 0)) * 1024 / (
                    batch * PMC_STEPS)
                # per candidate (round 5): the counted step's bytes over its candidates, without the dispatches whose
                # waves were context-saved (their bytes include the save, not kernel traffic); the median over those
                # dispatches of bytes / that dispatch's candidates (estimated by its share of the step's kernel time) is
                # kept beside it -- the two agree when the launches are alike
                bpc, bpc_med, bpc_all = 0.0, 0.0, 0.0
                for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
                    vals = passes.get(sub, {}).get(name)
                    ds = dur[k].get(sub, {})
                    tdur = sum(ds.get(d, 0) for d in (vals or {}))
                    if not vals or not tdur:
                        continue
                    cands = {d: batch * PMC_STEPS * ds[d] / tdur for d in vals if ds.get(d)}
                    clean = [d for d in cands if d not in saves.get(sub, [])]
                    bpc_all += sum(vals[d] for d in cands) * 1024 / sum(cands.values())
                    if not clean:     # every counted dispatch was context-saved: the figure includes the saves
                        per["hbm_no_clean_dispatch"] = True
                        clean = list(cands)
                    if clean:
                        bpc += sum(vals[d] for d in clean) * 1024 / sum(cands[d] for d in clean)
                        pcs = sorted(vals[d] * 1024 / cands[d] for d in clean)
                        m = len(pcs)
                        bpc_med += pcs[m // 2] if m % 2 else (pcs[m // 2 - 1] + pcs[m // 2]) / 2
                        per.setdefault("hbm_bytes_per_candidate_by_dispatch", {})[name] = pcs
                per["hbm_bytes_per_candidate_with_saves"] = bpc_all
                per["hbm_bytes_per_candidate_median"] = bpc_med
                per["hbm_bytes_per_candidate"] = bpc
        summ[k] = per
    out["counters"] = summ
    json.dump(out, open(dst + ".json", "w"), indent=1)
    return summ


if __name__ == "__main__":
    print(json.dumps(summarize(sys.argv[1], sys.argv[2]), indent=1))

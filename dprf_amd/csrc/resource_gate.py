#!/usr/bin/env python3
"""Build gate on the compiler's kernel resource report (hipcc -Rpass-analysis=kernel-resource-usage).

The Makefile compiles every kernel object with that remark enabled, writes the remarks to <obj>.res and runs
this script on them.  It fails the build when a kernel spills to scratch beyond its stated bound, so a
compiler-flag or source change that starts spilling cannot ship silently (round 2 shipped k_odt_kdf with
20 B/lane of scratch under the max-ilp scheduler: 1.46x its algorithmic HBM writes).

Usage: resource_gate.py [--expect k1,k2,...] <file.res>...   (one line per kernel; exit 1 on a violation)

The gate fails closed (round 4): a remark block without a ScratchSize line, a report with no kernel in
it, or an expected kernel (--expect, the Makefile passes each object's kernel families) missing from the report
all fail the build -- a changed remark format or a dropped -Rpass-analysis flag must not read as "0 B of scratch".
"""
import re
import subprocess
import sys

# Kernel name (demangled; an entry with template arguments wins over the bare name) -> the most scratch it may
# use, bytes/lane.  Every kernel must appear here: an unknown kernel fails the gate too.
SCRATCH_LIMIT = {
    # every kernel at 0 B/lane since round 3 (list-mode R6 had 16 until the persistent loop stopped holding its lane
    # index and the watchdog's 64-bit timestamp in registers: dprf_kernels_r6.hip opaque_lane, idle_t0 in LDS)
    "k_office_kdf": 0,
    "k_office_check": 0,
    "k_odt_kdf": 0,
    "k_odt_check": 0,
    "k_pdf_r5": 0,
    "k_pdf_r24": 0,
    "k_pdf_r6": 0,
    "k_long_prehash": 0,      # round 4: candidates longer than a list slot
    "k_spell_symbols": 0,     # round 6: symbol windows (dprf_search_symbols)
}


def parse(text):
    rows, cur = {}, None
    for ln in text.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", ln)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z][A-Za-z /\[\]]*?): (\S+) \[-Rpass-analysis", ln)
        if m and cur:
            rows[cur][m.group(1).strip()] = m.group(2)
    return rows


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.split("\n")
    except OSError:
        return {n: n for n in names}
    return {n: (out[i] if i < len(out) and out[i] else n) for i, n in enumerate(names)}


def main(argv):
    bad, expect, paths = [], set(), []
    it = iter(argv)
    for a in it:
        if a == "--expect":
            expect |= {x for x in next(it, "").split(",") if x}
        else:
            paths.append(a)
    seen = set()
    for path in paths:
        rows = parse(open(path).read())
        if not rows:
            bad.append("%s: no kernel in the resource report" % path)
        dem = demangle(list(rows))
        for mangled, r in rows.items():
            name = dem[mangled].split("(")[0]
            full = re.sub(r"^void ", "", name)
            seen.add(full.split("<")[0])
            if "ScratchSize [bytes/lane]" not in r:
                bad.append("%s (no ScratchSize remark)" % name)
                continue
            scratch = int(r["ScratchSize [bytes/lane]"])
            limit = SCRATCH_LIMIT.get(full.replace(" ", ""), SCRATCH_LIMIT.get(full.split("<")[0]))
            ok = limit is not None and scratch <= limit
            print("%-6s %-44s VGPRs %-4s scratch %-3d (limit %s) occupancy %s" % (
                "ok" if ok else "FAIL", name[:44], r.get("VGPRs"), scratch, "unknown kernel" if limit is None else limit,
                r.get("Occupancy [waves/SIMD]")))
            if not ok:
                bad.append(name)
    for k in sorted(expect - seen):
        bad.append("%s (expected, not in the report)" % k)
    if bad:
        sys.stderr.write("resource_gate: scratch above the stated bound, unknown or missing kernel, or no report: %s\n" % ", ".join(bad))
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))

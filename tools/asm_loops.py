#!/usr/bin/env python3
"""Static look at a hipcc -save-temps .s: for every kernel, list loops (backward branches) with their
instruction mix (VALU / SALU / LDS / VMEM / scratch).  Used to check that hot loops stay spill-free and
to count VALU instructions per iteration for the roofline accounting in DESIGN.md."""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    for ln in open(path):
        m = re.match(r"^(_Z\w+|\w+):\s*(;.*)?$", ln)
        if m and not ln.startswith(".L"):
            if cur:
                yield cur, body
            cur, body = m.group(1), []
        elif cur:
            body.append(ln.rstrip())
            if ln.startswith(".Lfunc_end"):
                yield cur, body
                cur, body = None, []


def classify(op):
    if op.startswith("scratch_") or (op.startswith("buffer_") and "store" in op):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def analyse(name, body, pat):
    if pat and not re.search(pat, name):
        return
    labels = {}
    ins = []
    for ln in body:
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        t = ln.strip()
        if not t or t.startswith((";", ".")):
            continue
        ins.append(t.split()[0])
    print("==", name[:90], "instructions:", len(ins))
    # recompute with branch targets
    idx = 0
    for ln in body:
        t = ln.strip()
        m = re.match(r"^(\.LBB\w+):", t)
        if m or not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] <= idx:
                seg = ins[labels[tgt]:idx + 1]
                c = Counter(classify(o) for o in seg)
                if len(seg) > 30:
                    print("   loop %s..%d: %d ins  valu=%d salu=%d lds=%d vmem=%d scratch=%d" % (
                        tgt, idx, len(seg), c["valu"], c["salu"], c["lds"], c["vmem"], c["scratch"]))
        idx += 1


if __name__ == "__main__":
    pat = sys.argv[2] if len(sys.argv) > 2 else None
    for n, b in kernels(sys.argv[1]):
        analyse(n, b, pat)

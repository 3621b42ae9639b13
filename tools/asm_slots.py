#!/usr/bin/env python3
"""Issue-slot cost of a kernel's hottest loop from a hipcc -save-temps .s, with the gfx950 VALU rates
measured by tools/valu_peak.hip (profiles/valu_issue_rates_r01.txt): full-rate ops 1 slot, half-rate 2,
v_bitop3 1 (measured full rate, round 5).  Usage: asm_slots.py file.s kernel_regex"""
import re
import sys
from collections import Counter

FULL = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_xor_b32", "v_and_b32", "v_or_b32", "v_not_b32",
        "v_lshrrev_b32", "v_ashrrev_i32", "v_lshlrev_b16", "v_mov_b32", "v_add_co_u32", "v_addc_co_u32",
        "v_sub_co_u32", "v_subb_co_u32"}
HALF_RATE_FACTOR = {"v_bitop3_b32": 1.0}   # full rate unless all three sources share a VGPR bank (round 5: profiles/vgpr_bank_r04.txt)


def cost(op):
    base = re.sub(r"_e(32|64)$", "", op)
    if base in FULL:
        return 1.0
    if base in HALF_RATE_FACTOR:
        return HALF_RATE_FACTOR[base]
    if base.startswith("v_cndmask"):
        return 2.0
    return 2.0


def loops(path, kpat):
    text = open(path).read().splitlines()
    out = []
    cur = None
    body = []
    for ln in text:
        m = re.match(r"^(\w+):\s*(;.*)?$", ln)
        if m and not ln.startswith(".L"):
            cur, body = m.group(1), []
            continue
        if cur and re.search(kpat, cur):
            body.append(ln)
        if ln.startswith(".Lfunc_end") and cur and re.search(kpat, cur):
            out.append((cur, body))
            cur = None
    return out


def analyse(name, body):
    labels, ins = {}, []
    for ln in body:
        t = ln.strip()
        m = re.match(r"^(\.LBB\w+):", t)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not t or t.startswith((";", ".")):
            continue
        ins.append(t.split()[0].rstrip(","))
    best = None
    for i, op in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            pass
    idx = 0
    for ln in body:
        t = ln.strip()
        if not t or t.startswith((";", ".")) or re.match(r"^\.LBB", t):
            continue
        op = t.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            if tgt in labels and labels[tgt] <= idx:
                seg = ins[labels[tgt]:idx + 1]
                v = [o for o in seg if o.startswith("v_")]
                if len(v) >= MINV and sum(1 for o in v if REQ in o) >= 50 and (best is None or len(v) < len(best[1])):
                    best = (tgt, v, seg)
        idx += 1
    if not best:
        return
    tgt, v, seg = best
    c = Counter(re.sub(r"_e(32|64)$", "", o) for o in v)
    slots = sum(cost(o) * n for o, n in c.items())
    print("%s\n  loop %s: %d VALU instr, %.0f issue slots, %d LDS, %d SALU" % (
        name[:80], tgt, len(v), slots, sum(1 for o in seg if o.startswith("ds_")), sum(1 for o in seg if o.startswith("s_"))))
    for o, n in c.most_common(14):
        print("     %5d x %-22s %.1f slots" % (n, o, n * cost(o)))


MINV = 400
REQ = "v_alignbit"

if __name__ == "__main__":
    if len(sys.argv) > 3:
        MINV = int(sys.argv[3])
    for n, b in loops(sys.argv[1], sys.argv[2]):
        analyse(n, b)

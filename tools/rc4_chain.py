#!/usr/bin/env python3
"""Critical path of one group (two KSA steps) of the generated RC4 key schedule (tools/gen_rc4_ksa_asm.py), per
schedule variant -- what VERDICT r3 #4 asked to see next to each A/B.

For a group q in the middle of the block (the compare constants from the VGPR, no inline constants) the script
builds the register dependencies of its instructions and takes the longest path from the arrival of W (the pair read
at the end of group q-1) to the ISSUE of the next pair read W' (whose arrival starts group q+1), i.e. the part of the
loop-carried chain that is not LDS latency.  Costs (cycles of one wave64 instruction on gfx950,
profiles/valu_issue_rates_r02.txt / vgpr_bank_r04.txt): half-rate VALU (v_add3, v_and_or, SDWA ops, v_cmp, v_perm) 4,
full-rate (v_add, v_xor, v_bitop3 with two source banks, v_cndmask_e32) 2, an LDS instruction 1 to issue.  The chain
then adds one LDS round trip (~120 cycles at 9 waves per CU, MI355X_MICROARCH.md's loaded latency) per group.

Usage: tools/rc4_chain.py [flags of gen_rc4_ksa_asm.py ...]   (no flags: the default schedule and every variant)
"""
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
GEN = os.path.join(HERE, "gen_rc4_ksa_asm.py")
HALF = ("v_add3_u32", "v_and_or_b32", "v_perm_b32", "v_lshl_or_b32")
VARIANTS = ["", "--and-or", "--ic4", "--split-add", "--jctr", "--early-v1", "--late-merge", "--early-read",
            "--salu-consts"]


def cost(op, line):
    if op.startswith("ds_"):
        return 1
    if op.startswith("s_"):
        return 1
    if "sdwa" in op or op.startswith("v_cmp") or op in HALF:
        return 4
    return 2


def group_lines(text, nk=16, q=60):
    m = re.search(r"#define RC4_KSA_ASM_%d \\\n(.*?)\n    \"\"" % nk, text, re.S)
    prog = [ln.strip()[1:-len('\\n\\t" \\')] for ln in m.group(1).splitlines()]
    # groups are delimited by the pair read "ds_read_u16 %1 ..., offset:<pos(2q+2)>"
    pos = lambda i: ((i >> 2) << 8) + (i & 3)
    reads = [k for k, ln in enumerate(prog) if ln.startswith("ds_read_u16") and ln.endswith("offset:%d" % pos(2 * q))]
    nxt = [k for k, ln in enumerate(prog) if ln.startswith("ds_read_u16") and ln.endswith("offset:%d" % pos(2 * q + 2))]
    assert reads and nxt, "group %d not found" % q
    return prog[reads[0] + 1: nxt[0] + 1]


def analyse(lines):
    ready = {"%1": 0}               # W arrives at t = 0
    t_issue = 0
    path = 0
    n_valu = n_lds = n_salu = 0
    issue_cycles = 0
    for ln in lines:
        op, _, rest = ln.partition(" ")
        if op == "s_waitcnt":
            continue
        args = [a.strip().split()[0] for a in rest.split(",") if a.strip()]
        c = cost(op, ln)
        issue_cycles += c
        if op.startswith("ds_"):
            n_lds += 1
        elif op.startswith("s_"):
            n_salu += 1
        else:
            n_valu += 1
        srcs = args if op.startswith("ds_write") else args[1:]
        dst = None if op.startswith("ds_write") else (args[0] if args else None)
        if "dst_unused:UNUSED_PRESERVE" in ln and dst:
            srcs = srcs + [dst]
        if op.startswith("v_cndmask") or op.startswith("v_cmp"):
            srcs = srcs + ["vcc"]
        start = max([ready.get(s, 0) for s in srcs if s.startswith("%") or s == "vcc"] + [0])
        done = start + c
        if op.startswith("v_cmp"):
            ready["vcc"] = done
        elif dst and not op.startswith("ds_read"):
            ready[dst] = done
        if op.startswith("ds_read_u16"):
            path = start          # the next pair read issues once its own inputs (the stores before it, in order) can
            # the LDS pipe keeps program order: W' cannot issue before the S[j] stores ahead of it
        if op.startswith("ds_write") or op.startswith("ds_read"):
            ready["__lds"] = max(ready.get("__lds", 0), start)
    path = max(path, ready.get("__lds", 0))
    return path, n_valu, n_lds, n_salu, issue_cycles


def main():
    flags = sys.argv[1:] or VARIANTS
    print("%-14s %22s %6s %5s %5s %14s" % ("variant", "chain to W' issue (cy)", "VALU", "LDS", "SALU", "issue cy/group"))
    for f in flags:
        text = subprocess.run([sys.executable, GEN] + f.split(), capture_output=True, text=True, check=True).stdout
        path, nv, nl, ns, ic = analyse(group_lines(text))
        print("%-14s %22d %6d %5d %5d %14d" % (f or "(default)", path, nv, nl, ns, ic))


if __name__ == "__main__":
    main()

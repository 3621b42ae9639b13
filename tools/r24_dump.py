#!/usr/bin/env python3
"""Trace a PDF R3/R4 verdict through k_pdf_r24 on the GPU (round 5, VERDICT r4 "next" #1).

Runs verify_list on one verdict table of tests/golden (default pdf_testdoc_r4) with a libdprf built with
-DDPRF_DEBUG_R24 (DPRF_LIB=<that .so>), reads the kernel's debug words (dprf_debug_r24_read, dprf_kernels.hip) and
replays the reference's R3/R4 chain on the CPU -- MD5 key derivation (pdf_password_verifier.c:136-158, 352-402) and
c = RC4(key ^ x, c) for x = 0..19 (:164-176) -- with hashlib and a plain RC4.  Prints, per lane, the first thing that
differs: the key, lane 0's S-box after a pass's KSA, or the data words after a pass.

Usage: DPRF_LIB=build/ab/libdprf_dbg.so python3 tools/r24_dump.py [table] """
import ctypes
import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))

PAD = bytes.fromhex("28bf4e5e4e758a4164004e56fffa01082e2e00b6d0683e802f0ca9fe6453697a")


def rc4_ksa(key):
    S = list(range(256))
    j = 0
    for i in range(256):
        j = (j + S[i] + key[i % len(key)]) & 0xff
        S[i], S[j] = S[j], S[i]
    return S


def rc4_stream(S, n):
    S = S[:]
    i = j = 0
    out = []
    for _ in range(n):
        i = (i + 1) & 0xff
        j = (j + S[i]) & 0xff
        S[i], S[j] = S[j], S[i]
        out.append(S[(S[i] + S[j]) & 0xff])
    return bytes(out)


def ref_chain(f, pw):
    """(key, [S-box after KSA of pass x], [data after pass x]) for the R3/R4 user-password check"""
    R, length, P, meta = int(f[2]), int(f[3]), int(f[4]), int(f[5])
    ID, O = bytes.fromhex(f[7]), bytes.fromhex(f[11])
    n = length // 8
    m = (pw[:32] + PAD)[:32] + O + struct.pack("<i", P) + ID
    if R >= 4 and not meta:
        m += b"\xff\xff\xff\xff"
    h = hashlib.md5(m).digest()
    for _ in range(50):
        h = hashlib.md5(h[:n]).digest()
    key = h[:n]
    c = hashlib.md5(PAD + ID).digest()
    boxes, datas = [], []
    for x in range(20):
        kx = bytes(b ^ x for b in key)
        S = rc4_ksa(kx if n == 5 else (kx + bytes(16))[:16])
        boxes.append(S)
        c = bytes(a ^ b for a, b in zip(c, rc4_stream(S, 16)))
        datas.append(c)
    return key, boxes, datas


def main():
    table = sys.argv[1] if len(sys.argv) > 1 else "pdf_testdoc_r4"
    from dprf_amd import _lib, brute_force as bf
    g = os.path.join(HERE, "..", "tests", "golden")
    streams = json.load(open(os.path.join(g, "streams.json")))
    verdicts = json.load(open(os.path.join(g, "verdicts.json")))
    fields = bf.parse_verification_data(streams[table]["stream"])
    cands = [p for p, _ in verdicts[table]]
    want = [i for i, (_, v) in enumerate(verdicts[table]) if v]
    c = _lib.Context(fields)
    hits, nh, st = c.verify_list(cands)
    print("table %s: %d candidates, hits %s, want %s -> %s" % (table, len(cands), hits, want,
                                                                "OK" if hits == want else "WRONG"))
    L = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_uint32 * 11784)()
    rc = L.dprf_debug_r24_read(buf, 11784)
    assert rc == 0, rc
    w = list(buf)
    print("sweeps run:", w[11776])
    n = int(fields[3]) // 8
    bad = 0
    for lane, pw in enumerate(cands[:64]):
        key, boxes, datas = ref_chain(fields, pw.encode() if isinstance(pw, str) else pw)
        hk = struct.pack("<4I", *w[4 * lane:4 * lane + 4])[:n]
        if hk != key:
            print("lane %d %r: KEY differs: gpu %s ref %s" % (lane, pw, hk.hex(), key.hex()))
            bad += 1
            continue
        if lane == 0:
            for x in range(20):
                gb = b"".join(struct.pack("<I", w[10496 + 64 * x + k]) for k in range(64))
                if list(gb) != boxes[x]:
                    d = [i for i in range(256) if gb[i] != boxes[x][i]]
                    print("lane 0 pass %d: S-box after the KSA differs at %d positions, first S[%d] gpu %d ref %d"
                          % (x, len(d), d[0], gb[d[0]], boxes[x][d[0]]))
                    bad += 1
                    break
        for full in range(w[11776]):
            for x in range(20):
                o = 256 + ((full * 20 + x) * 64 + lane) * 4
                gd = struct.pack("<4I", *w[o:o + 4])
                nb = 16 if full else 2
                if gd[:nb] != datas[x][:nb]:
                    print("lane %d %r sweep %d pass %d: data differs gpu %s ref %s"
                          % (lane, pw, full, x, gd[:nb].hex(), datas[x][:nb].hex()))
                    bad += 1
                    break
            else:
                continue
            break
    print("R24DUMP: %s (%d lanes checked)" % ("all lanes == the CPU chain" if not bad else "%d differences" % bad,
                                                min(64, len(cands))))
    return 0 if (hits == want and not bad) else 1


if __name__ == "__main__":
    sys.exit(main())

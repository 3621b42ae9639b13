#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE verifiers.

Runs only in the build container (needs /root/reference and oracle/_ref from `make -f oracle/ref.mk`).
Every verdict, hit set and intermediate recorded here is the output of the reference's own compiled
verifier executables, invoked with exactly the argv brute_force.py builds (brute_force.py:163-197).
Synthetic documents are constructed with the oracle's primitives and then ACCEPTED only if the
reference verifier returns 1 for the intended password.

    python tests/golden/make_golden.py [--slow]

Outputs (committed):
  streams.json        name -> {stream, password, source}
  verdicts.json       name -> [[candidate, reference exit code], ...]
  hitsets.json        name -> {charset, pwlen, start, count, hits: [indices]}  (full keyspace scans)
  intermediates.json  name -> {password, lines: {label: hex}}  (reference -v output)
"""
import argparse
import json
import os
import random
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)
import pyoracle as O  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref")
REFSRC = "/root/reference"
ENV = dict(os.environ, OPENSSL_CONF=os.path.join(REPO, "oracle", "openssl_legacy.cnf"))
LOWER = "abcdefghijklmnopqrstuvwxyz"
PDF_PAD = bytes.fromhex("28bf4e5e4e758a4164004e56fffa01082e2e00b6d0683e802f0ca9fe6453697a")


def ref_argv(fields, pw):
    """The argv brute_force.py builds per candidate (_call_*_core, brute_force.py:163-197)."""
    f = fields
    if f[0] == "office":
        return [REF + "/msoffcrypto", pw, f[5], f[4], f[6], str(len(f[6]) // 2), f[7], str(len(f[7]) // 2),
                str(f[3]), str(f[2])]
    if f[0] == "odt":
        return [REF + "/odt", pw, f[2], f[3], f[4], f[5], str(f[6])]
    if f[0] == "pdf":
        return [REF + "/pdf", pw] + [str(x) for x in f[1:12]]
    raise ValueError(f[0])


def ref_verdict(fields, pw):
    return subprocess.run(ref_argv(fields, pw), env=ENV, stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL).returncode


def ref_verbose(fields, pw):
    out = subprocess.run(ref_argv(fields, pw) + ["-v"], env=ENV, capture_output=True).stdout
    lines = {}
    for ln in out.decode("latin-1").splitlines():
        m = re.match(r"\s*([^:]+):\s*([0-9a-f]+)\s*$", ln)
        if m:
            lines[m.group(1).strip()] = m.group(2)
    return lines


def rnd_bytes(rng, n):
    while True:
        b = bytes(rng.getrandbits(8) for _ in range(n))
        if b[0] != 0:          # str_to_uchar drops a leading 00 byte
            return b


def aes_cbc_encrypt(key, iv, pt):
    out, prev = b"", iv
    for i in range(0, len(pt), 16):
        blk = bytes(a ^ b for a, b in zip(pt[i:i + 16], prev))
        prev = O.aes_encrypt_block(key, blk)
        out += prev
    return out


# ---------------------------------------------------------------- synthetic document streams
def synth_office(rng, pw, name="synth.docx"):
    salt = rnd_bytes(rng, 16)
    dummy = "%s:$office$*2007*20*128*16*%s*%s*%s" % (name, salt.hex(), rnd_bytes(rng, 16).hex(), rnd_bytes(rng, 32).hex())
    key = O.Ctx(dummy).intermediates(pw)[40:56]
    while True:
        verifier = rnd_bytes(rng, 16)
        vh = O.sha1(verifier) + bytes(12)
        ev = O.aes_encrypt_block(key, verifier)
        evh = O.aes_encrypt_block(key, vh[:16]) + O.aes_encrypt_block(key, vh[16:])
        if ev[0] and evh[0]:
            break
    return "%s:$office$*2007*20*128*16*%s*%s*%s" % (name, salt.hex(), ev.hex(), evh.hex())


def synth_odt(rng, pw, experimental, name="synth.odt"):
    salt, iv = rnd_bytes(rng, 16), rnd_bytes(rng, 16)
    dummy = "%s:$odt$*1.2*%s*%s*%s*%s*16" % (name, rnd_bytes(rng, 32).hex(), iv.hex(), salt.hex(), rnd_bytes(rng, 16).hex())
    key = O.Ctx(dummy).intermediates(pw)[32:64]
    while True:
        if experimental:
            pt = b"\x03\x00" + bytes(rng.getrandbits(8) for _ in range(14))
        else:
            pt = bytes(rng.getrandbits(8) for _ in range(1312))
        enc = aes_cbc_encrypt(key, iv, pt)
        checksum = O.sha256(pt[:1024])
        if enc[0] and checksum[0]:
            break
    return "%s:$odt$*1.2*%s*%s*%s*%s*%d" % (name, checksum.hex(), iv.hex(), salt.hex(), enc.hex(), len(enc))


def synth_pdf(rng, pw, V, R, length, P, meta, name="synth.pdf"):
    id_ = rnd_bytes(rng, 16)
    if R >= 5:
        vsalt, ksalt = rnd_bytes(rng, 8), rnd_bytes(rng, 8)
        o = rnd_bytes(rng, 48)
        dummy_u = rnd_bytes(rng, 32) + vsalt + ksalt
        head = "%s:$pdf$*%d*%d*%d*%d*%d*16*%s*48*" % (name, V, R, length, P, meta, id_.hex())
        h = O.Ctx(head + dummy_u.hex() + "*48*" + o.hex()).intermediates(pw)[:32]
        u = h + vsalt + ksalt
        assert u[0] != 0, "retry seed"
        return head + u.hex() + "*48*" + o.hex()
    o = rnd_bytes(rng, 32)
    head = "%s:$pdf$*%d*%d*%d*%d*%d*16*%s*32*" % (name, V, R, length, P, meta, id_.hex())
    ct = O.Ctx(head + rnd_bytes(rng, 32).hex() + "*32*" + o.hex()).intermediates(pw)[48:80]
    u = ct if R == 2 else ct[:16] + bytes(16)
    assert u[0] != 0, "retry seed"
    return head + u.hex() + "*32*" + o.hex()


def build_streams(rng):
    s = {}
    # reference test documents
    off = subprocess.run([sys.executable, REFSRC + "/src/ms-offcrypto-impl/office2john.py",
                          REFSRC + "/test/files/ms/password.docx"], capture_output=True, text=True).stdout.strip()
    s["office_testdoc"] = dict(stream=off, password="password",
                               source="reference office2john.py (py3 output == py2 for Standard Encryption)")
    from dprf_amd.parsers import odt2hashes
    s["odt_testdoc_e"] = dict(stream=odt2hashes.get_hashes(REFSRC + "/test/files/odt/password.odt", True),
                              password="password", source="dprf_amd.parsers.odt2hashes -e (== SURVEY Appendix A)")
    s["odt_testdoc_std"] = dict(stream=odt2hashes.get_hashes(REFSRC + "/test/files/odt/password.odt", False),
                                password="password", source="dprf_amd.parsers.odt2hashes (server.py:285 path)")
    s["pdf_testdoc_r4"] = dict(
        stream="password_1.7_v4_r4.pdf:$pdf$*4*4*128*-3904*1*16*711f273e163f024fb95b1de8541e9148*32*"
               "9984b2ecfa4da0c94eea1c75849a245200000000000000000000000000000000*32*"
               "408b37bcf12da873d7f2840f3c1b917a023961ded4c8164d38e46e9655e66775",
        password="password", source="pdf2john.py with py2 semantics (SURVEY Appendix A)")
    s["pdf_testdoc_r2"] = dict(
        stream="password_1.3_v1_r2.pdf:$pdf$*1*2*40*-64*1*16*5f1f3a5cf9db56448dac58ede8ac3183*32*"
               "02b69f455c9c71ad298adc1c71aa11d56eeaa7c3224133cffc68e670a2136d01*32*"
               "842e9696ecdf13a829f3b63c5b9614cc6254b7e0385b247bab90a508179c0340",
        password="password", source="pdf2john.py with py2 semantics (SURVEY Appendix A)")
    # synthetic documents (seed 0xD9F); short passwords so full keyspace scans contain the hit
    s["office_synth_ok"] = dict(stream=synth_office(rng, "ok"), password="ok", source="synthetic")
    s["office_synth_dprf"] = dict(stream=synth_office(rng, "dprf"), password="dprf", source="synthetic (config 1 positive)")
    s["odt_synth_e_ab"] = dict(stream=synth_odt(rng, "ab", True), password="ab", source="synthetic -e")
    s["odt_synth_std_zq"] = dict(stream=synth_odt(rng, "zq", False), password="zq", source="synthetic standard")
    s["odt_synth_std_alnum"] = dict(stream=synth_odt(rng, "Q7x", False), password="Q7x", source="synthetic standard")
    s["pdf_synth_r2_key"] = dict(stream=synth_pdf(rng, "key", 1, 2, 40, -64, 1), password="key", source="synthetic")
    s["pdf_synth_r3_l128_abc"] = dict(stream=synth_pdf(rng, "abc", 2, 3, 128, -1028, 1), password="abc", source="synthetic")
    s["pdf_synth_r3_l40_cab"] = dict(stream=synth_pdf(rng, "cab", 2, 3, 40, -1028, 1), password="cab", source="synthetic")
    s["pdf_synth_r4_meta0_dog"] = dict(stream=synth_pdf(rng, "dog", 4, 4, 128, -3904, 0), password="dog", source="synthetic")
    s["pdf_synth_r5_cat"] = dict(stream=synth_pdf(rng, "cat", 5, 5, 256, -1028, 1), password="cat", source="synthetic")
    s["pdf_synth_r6_ox"] = dict(stream=synth_pdf(rng, "ox", 5, 6, 256, -1028, 1), password="ox", source="synthetic")
    s["pdf_synth_r6_long"] = dict(stream=synth_pdf(rng, "Tr0ub4dor&3-correct-horse", 5, 6, 256, -4, 1),
                                  password="Tr0ub4dor&3-correct-horse", source="synthetic (long password)")
    s["pdf_synth_r5_alnum"] = dict(stream=synth_pdf(rng, "x9Z", 5, 5, 256, -1028, 1), password="x9Z", source="synthetic")
    s["pdf_synth_r4_alnum"] = dict(stream=synth_pdf(rng, "Zz9", 4, 4, 128, -1028, 1), password="Zz9", source="synthetic")
    # every stream must be accepted by the reference for its password
    for name, d in s.items():
        f = O.split_stream(d["stream"])
        rc = ref_verdict(f, d["password"])
        assert rc == 1, (name, rc)
    return s


def candidates_for(pw, rng):
    c = [pw, pw[:-1] or "x", pw + "a", pw.upper(), pw[::-1] + "q", "Password", "password", "passwore",
         "test", "a", "zzzzzzzz", "_dummy", "hunter2", "correcthorse", "été", "p@ss w0rd!",
         "A" * 31, "B" * 32, "C" * 33, "0123456789abcdef0123456789"]
    for _ in range(12):
        n = rng.randint(1, 12)
        c.append("".join(rng.choice(LOWER + "0123456789ABC") for _ in range(n)))
    seen, out = set(), []
    for x in c:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def index_to_pw(idx, cs, n):
    return O.index_to_password(idx, cs, n)


def ref_hitset(fields, cs, n, start, count, workers=8):
    def one(i):
        return i if ref_verdict(fields, index_to_pw(i, cs, n)) else None
    with ThreadPoolExecutor(workers) as ex:
        res = ex.map(one, range(start, start + count), chunksize=64)
        return [i for i in res if i is not None]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slow", action="store_true", help="also scan ODT -e [a-z]^4 with the reference (~5 min)")
    a = ap.parse_args()
    rng = random.Random(0xD9F)
    streams = build_streams(rng)
    json.dump(streams, open(os.path.join(HERE, "streams.json"), "w"), indent=1)

    verdicts = {}
    for name, d in streams.items():
        f = O.split_stream(d["stream"])
        cands = candidates_for(d["password"], rng)
        if f[0] == "office":   # empty/invalid UTF-8 is undefined behaviour in the reference (iconv path)
            cands = [c for c in cands if c]
        verdicts[name] = [[c, ref_verdict(f, c)] for c in cands]
        print(name, sum(v for _, v in verdicts[name]), "hits of", len(cands), flush=True)
    json.dump(verdicts, open(os.path.join(HERE, "verdicts.json"), "w"), indent=0)

    scans = [  # (stream, charset, pwlen)
        ("office_synth_ok", LOWER, 2), ("office_testdoc", LOWER, 2),
        ("odt_synth_e_ab", LOWER, 2), ("odt_synth_std_zq", LOWER, 2), ("odt_testdoc_e", LOWER, 3),
        ("pdf_testdoc_r2", LOWER, 3), ("pdf_synth_r2_key", LOWER, 3), ("pdf_synth_r3_l128_abc", LOWER, 3),
        ("pdf_synth_r3_l40_cab", LOWER, 3), ("pdf_synth_r4_meta0_dog", LOWER, 3), ("pdf_testdoc_r4", LOWER, 3),
        ("pdf_synth_r5_cat", LOWER, 3), ("pdf_synth_r6_ox", LOWER, 2),
    ]
    if a.slow:
        scans.append(("odt_testdoc_e", LOWER, 4))
    hitsets = {}
    for name, cs, n in scans:
        f = O.split_stream(streams[name]["stream"])
        hits = ref_hitset(f, cs, n, 0, len(cs) ** n)
        key = "%s/%s^%d" % (name, "lower" if cs == LOWER else cs, n)
        hitsets[key] = dict(stream=name, charset=cs, pwlen=n, start=0, count=len(cs) ** n, hits=hits)
        print(key, hits, flush=True)
    old = os.path.join(HERE, "hitsets.json")
    if os.path.exists(old) and not a.slow:   # keep a previously generated slow scan
        prev = json.load(open(old))
        for k, v in prev.items():
            hitsets.setdefault(k, v)
    json.dump(hitsets, open(old, "w"), indent=1)

    inter = {}
    for name, d in streams.items():
        f = O.split_stream(d["stream"])
        inter[name] = dict(password=d["password"], lines=ref_verbose(f, d["password"]))
    json.dump(inter, open(os.path.join(HERE, "intermediates.json"), "w"), indent=1)


if __name__ == "__main__":
    main()

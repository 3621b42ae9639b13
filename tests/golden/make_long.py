#!/usr/bin/env python3
"""Golden verdicts for LONG candidates (round 4), from the REFERENCE verifiers.

The list slots of the kernels hold 64 bytes; the reference hashes any strlen(password) (odt...c:79), converts any
length to UTF-16LE (msoffcrypto...c:75, 287-296), truncates PDF R5 at 127 (pdf...c:197-206) and takes R6 whole
into data[(128 + 64 + 48) * 64] (:117, :228).  This records, for synthetic documents whose passwords are long
themselves, the reference's exit code for candidates at the boundary lengths 64/65/119/120/127/128/176/177/200 and
multi-byte UTF-8 (2-, 3- and 4-byte sequences, i.e. UTF-16 surrogate pairs for Office).  An exit code of -6 is the
reference aborting (R6 over 176 bytes: "stack smashing detected"), which brute_force.py would count as "found"
(brute_force.py:140); the library returns DPRF_E_DOMAIN for those instead.

Runs only in the build container (needs /root/reference built into oracle/_ref by `make -f oracle/ref.mk`):
    python tests/golden/make_long.py          -> tests/golden/long_verdicts.json
"""
import json
import os
import random
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as G  # noqa: E402

O = G.O
LENGTHS = (64, 65, 119, 120, 127, 128, 176, 177, 200)


def ref_code(fields, pw):
    r = subprocess.run(G.ref_argv(fields, pw), env=G.ENV, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return r.returncode


def rnd_text(rng, n, alphabet="abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789-_!"):
    return "".join(rng.choice(alphabet) for _ in range(n))


def candidates(rng, pw):
    """The password, its near misses, and candidates at every boundary length (ASCII and multi-byte UTF-8)."""
    b = pw.encode()
    c = [pw, pw[:-1], pw + "x", pw[1:], pw[::-1], pw.upper() if pw.upper() != pw else pw.lower()]
    for n in LENGTHS:
        c.append(rnd_text(rng, n))
        c.append((pw * (n // max(1, len(pw)) + 1))[:n])          # shares the password's prefix
    # multi-byte UTF-8: 2-byte (é), 3-byte (日), 4-byte (😀: a surrogate pair in UTF-16)
    for unit in ("é", "日", "😀", "aé日😀"):
        for n in (16, 33, 40, 70):
            c.append((unit * n)[:n] if len(unit) == 1 else (unit * (n // 4 + 1))[:n])
    c.append("pässwörd-" * 9)
    c.append(pw + "é")
    if len(b) >= 127:                                             # R5 truncation: equal first 127 bytes match
        c.append(pw[:127] + "tail-after-127")
    seen, out = set(), []
    for x in c:
        if x and x not in seen and "\x00" not in x:
            seen.add(x)
            out.append(x)
    return out


def main():
    rng = random.Random(0x10D6)
    docs = {
        "office_long_ascii70": ("office", rnd_text(rng, 70)),
        "office_long_utf8": ("office", "pässwörd-日本語-😀-" * 4),
        "odt_long_std_100": ("odt_std", rnd_text(rng, 100)),
        "odt_long_e_200": ("odt_e", rnd_text(rng, 200)),
        "pdf_r4_long40": ("pdf4", rnd_text(rng, 40)),
        "pdf_r5_long90": ("pdf5", rnd_text(rng, 90)),
        "pdf_r5_long127": ("pdf5", rnd_text(rng, 127)),
        "pdf_r5_long150": ("pdf5", rnd_text(rng, 150)),
        "pdf_r6_long100": ("pdf6", rnd_text(rng, 100)),
        "pdf_r6_long176": ("pdf6", rnd_text(rng, 176)),
        "pdf_r6_utf8": ("pdf6", "日本語のパスワード-" * 5),
    }
    out = {}
    for name, (kind, pw) in docs.items():
        if kind == "office":
            s = G.synth_office(rng, pw, name + ".docx")
        elif kind == "odt_std":
            s = G.synth_odt(rng, pw, False, name + ".odt")
        elif kind == "odt_e":
            s = G.synth_odt(rng, pw, True, name + ".odt")
        elif kind == "pdf4":
            s = G.synth_pdf(rng, pw, 4, 4, 128, -3904, 1, name + ".pdf")
        elif kind == "pdf5":
            s = G.synth_pdf(rng, pw, 5, 5, 256, -1028, 1, name + ".pdf")
        else:
            s = G.synth_pdf(rng, pw, 5, 6, 256, -1028, 1, name + ".pdf")
        f = O.split_stream(s)
        assert ref_code(f, pw) == 1, (name, "the reference must accept the document's own password")
        cands = candidates(rng, pw)
        table = [[c, ref_code(f, c)] for c in cands]
        out[name] = dict(stream=s, password=pw, verdicts=table)
        codes = {}
        for _, v in table:
            codes[v] = codes.get(v, 0) + 1
        print(name, len(pw.encode()), "bytes;", len(table), "candidates; exit codes", codes, flush=True)
    json.dump(out, open(os.path.join(HERE, "long_verdicts.json"), "w"), indent=0, ensure_ascii=False)


if __name__ == "__main__":
    main()

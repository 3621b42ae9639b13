#!/usr/bin/env python3
"""Generate the self-made encrypted documents in tests/golden/docs/ and their reference fixtures.

Runs only in the build container (needs /root/reference and oracle/_ref from `make -f oracle/ref.mk`):

    python tests/golden/make_docs.py

For every document written by tests/docgen.py (fixed seeds):
  * the verifier stream our parsers (dprf_amd/parsers) produce -- and, for Office and PDF, the stream the
    REFERENCE's own office2john.py / pdf2john.py print for the same file (they run under Python 3 for these
    inputs), which must be identical;
  * reference verdicts: the reference verifier executables (oracle/_ref, compiled from /root/reference)
    run with exactly the argv brute_force.py builds, for the password and wrong candidates;
  * the full [a-z]^3 hit set of the reference verify() (in-process oracle/_ref/libref_*.so), i.e. every
    candidate of the keyspace the reference accepts.
A document is kept only if the reference accepts its password.  Output: tests/golden/docs.json.
"""
import json
import multiprocessing as mp
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(HERE))
import docgen  # noqa: E402
from dprf_amd.brute_force import _index_to_password  # noqa: E402
from dprf_amd.parsers import odt2hashes, office2john, pdf2john  # noqa: E402

sys.path.insert(0, HERE)
from make_golden import ENV, ref_argv  # noqa: E402

DOCS = os.path.join(HERE, "docs")
REFSRC = "/root/reference/src"
LOWER = "abcdefghijklmnopqrstuvwxyz"

SPECS = [
    # name, writer, password, kwargs
    ("office_std.docx", "docx", "key", {}),
    ("odf12.odt", "odt", "odf", {}),
    ("pdf_r2.pdf", "pdf", "cat", {"R": 2, "length": 40, "P": -64}),
    ("pdf_r3_l128.pdf", "pdf", "dog", {"R": 3, "length": 128, "P": -1028}),
    ("pdf_r3_l40.pdf", "pdf", "owl", {"R": 3, "length": 40, "P": -1340}),
    ("pdf_r4.pdf", "pdf", "fox", {"R": 4, "length": 128, "P": -3904}),
    ("pdf_r4_meta0.pdf", "pdf", "elk", {"R": 4, "length": 128, "P": -3904, "meta": False}),
    ("pdf_r5.pdf", "pdf", "bee", {"R": 5, "P": -1028}),
    ("pdf_r6.pdf", "pdf", "yak", {"R": 6, "P": -4}),
]
WRONG = ["Key", "ke", "keyy", "password", "zzz"]


def fields_of(stream):
    import contextlib
    import io
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def ref_verdict(fields, pw):
    return subprocess.run(ref_argv(fields, pw), env=ENV, stdout=subprocess.DEVNULL,
                          stderr=subprocess.DEVNULL).returncode


def _scan(job):
    fields, lo, hi = job
    sys.path.insert(0, REPO)
    import bench
    fn = bench.ref_callable(fields)
    return [i for i in range(lo, hi) if fn(_index_to_password(i, LOWER, 3).encode()) == 1]


def ref_hitset(fields, pool):
    n = 26 ** 3
    step = 256
    parts = pool.map(_scan, [(fields, lo, min(n, lo + step)) for lo in range(0, n, step)])
    return sorted(i for p in parts for i in p)


def ref_parser(kind, path):
    script = {"docx": REFSRC + "/ms-offcrypto-impl/office2john.py", "pdf": REFSRC + "/pdf-impl/pdf2john.py"}.get(kind)
    if script is None:
        return None
    out = subprocess.run([sys.executable, script, path], capture_output=True, text=True, cwd=DOCS)
    return out.stdout.strip() or None


def main():
    os.makedirs(DOCS, exist_ok=True)
    out = {}
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        for seed, (name, kind, pw, kw) in enumerate(SPECS, start=101):
            path = os.path.join(DOCS, name)
            if kind == "docx":
                docgen.write_docx(path, pw, seed)
                streams = {"std": office2john.get_hash(path)}
            elif kind == "odt":
                docgen.write_odt(path, pw, seed)
                streams = {"std": odt2hashes.get_hashes(path, False), "e": odt2hashes.get_hashes(path, True)}
            else:
                docgen.write_pdf(path, pw, seed, **kw)
                streams = {"std": pdf2john.get_hash(path)}
            rp = ref_parser(kind, path)
            if rp is not None and rp != streams["std"]:
                raise SystemExit("%s: reference parser disagrees:\n  ours %s\n  ref  %s" % (name, streams["std"], rp))
            entry = {"file": name, "kind": kind, "password": pw, "seed": seed, "kwargs": kw,
                     "reference_parser_agrees": rp is not None, "streams": {}}
            for sk, stream in streams.items():
                f = fields_of(stream)
                verdicts = [[c, ref_verdict(f, c)] for c in [pw] + WRONG]
                if verdicts[0][1] != 1:
                    raise SystemExit("%s/%s: the reference verifier rejects the password" % (name, sk))
                hits = ref_hitset(f, pool)
                entry["streams"][sk] = {"stream": stream, "verdicts": verdicts,
                                        "hitset": {"charset": LOWER, "pwlen": 3, "hits": hits}}
                print("%-18s %-3s hits %s" % (name, sk, [_index_to_password(i, LOWER, 3) for i in hits]), flush=True)
            out[name] = entry
    with open(os.path.join(HERE, "docs.json"), "w") as fo:
        json.dump(out, fo, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

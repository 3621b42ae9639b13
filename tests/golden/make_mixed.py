#!/usr/bin/env python3
"""Golden candidates for a list that mixes SHORT (slot-sized, <= 64 bytes) and LONG hits on ONE document (round 5,
ADVICE r4): the ODF `-e` stream of odt_long_e_200 (long_verdicts.json), whose 2-byte check (odt...c:98-101) accepts
about 2^-16 of all candidates.  Its password is 200 bytes (a long hit); this script searches short alnum candidates
with the CPU oracle until it has found short false positives, and records the REFERENCE verifier's exit code for each
(1 = the reference accepts it, so brute_force.py would report it as found).

Runs only in the build container (needs oracle/_ref built by `make -f oracle/ref.mk` and oracle/_build):
    python tests/golden/make_mixed.py          -> tests/golden/mixed_verdicts.json
"""
import json
import multiprocessing as mp
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import make_long as ML  # noqa: E402

ALNUM = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"
DOC = "odt_long_e_200"
WANT = 3


def _cands(seed, n):
    rng = random.Random(seed)
    return ["".join(rng.choice(ALNUM) for _ in range(rng.choice((5, 6, 7, 8)))) for _ in range(n)]


def _search(args):
    stream, seed, n = args
    import pyoracle
    ctx = pyoracle.Ctx(stream)
    return [c for c in _cands(seed, n) if ctx.verify(c) == 1]


def main():
    long_v = json.load(open(os.path.join(HERE, "long_verdicts.json")))
    d = long_v[DOC]
    from dprf_amd import brute_force as bf   # noqa: F401  (only the parser's field split is used below)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        fields = bf.parse_verification_data(d["stream"])
    found = []
    seed = 0
    with mp.get_context("spawn").Pool(8) as pool:
        while len(found) < WANT:
            for hits in pool.map(_search, [(d["stream"], seed + k, 4096) for k in range(8)]):
                found.extend(hits)
            seed += 8
    found = found[:WANT]
    codes = {c: ML.ref_code(fields, c) for c in found + [d["password"]]}
    assert all(v == 1 for v in codes.values()), codes
    out = {"document": DOC, "stream": d["stream"], "long_hit": d["password"], "short_hits": found,
           "reference_exit_codes": codes,
           "note": "short_hits: alnum candidates the ODF -e 2-byte check accepts (odt_password_verifier.c:98-101), found "
                   "with the CPU oracle and confirmed by the reference verifier (exit code 1)"}
    json.dump(out, open(os.path.join(HERE, "mixed_verdicts.json"), "w"), indent=1)
    print(json.dumps(out)[:400])


if __name__ == "__main__":
    sys.path.insert(0, os.path.join(HERE, "..", ".."))
    main()

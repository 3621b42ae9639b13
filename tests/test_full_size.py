"""BASELINE.json's configs at their full keyspace sizes, through position properties that do not need the
whole space scanned: a self-generated document (tests/docgen.py) whose password sits deep in the config's
keyspace -- past 2^32 for the alnum^7 and lowercase^8 spaces (the u64 enumeration of brute_force.py:199-219
and of the server's global order), or at its very last index -- is searched in range mode over a window
around that index at the config's own charset and length.  The lowest hit must be the planted index, and
every hit the GPU reports must verify on the oracle (the CPU restatement of the reference verifiers).
"""
import os
import tempfile

import pytest

LOWER = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWER + LOWER.upper() + "0123456789"

# (config, writer kind, writer kwargs, charset, password, window)
CASES = [
    ("configs0-office-pr8", "docx", {}, LOWER, "pwzqxkmv", 1 << 19),
    ("configs1-odt-alnum6", "odt", {}, ALNUM, "Zx9Qa7", 1 << 22),
    ("configs2-pdf-r4-alnum7", "pdf", {"R": 4, "length": 128}, ALNUM, "q7ZpL02", 1 << 24),
    ("configs2-pdf-r3-alnum7-last", "pdf", {"R": 3, "length": 128}, ALNUM, "9999999", 1 << 24),
    ("configs3-pdf-r6-lower6", "pdf", {"R": 6, "length": 256}, LOWER, "zyxwvu", 1 << 19),
    ("pdf-r2-alnum7", "pdf", {"R": 2, "length": 40}, ALNUM, "Mo3kV9b", 1 << 26),
    ("pdf-r5-alnum7-first", "pdf", {"R": 5, "length": 256}, ALNUM, "aaaaaaa", 1 << 26),
]


def index_of(pw, cs):
    """itertools.product order (brute_force.py:205): the last character varies fastest."""
    i = 0
    for ch in pw:
        i = i * len(cs) + cs.index(ch)
    return i


def word(i, cs, n):
    out = []
    for _ in range(n):
        i, r = divmod(i, len(cs))
        out.append(cs[r])
    return "".join(reversed(out))


def _doc_streams(t, kind, kw, pw, seed):
    import docgen
    from dprf_amd.parsers import odt2hashes, office2john, pdf2john
    path = os.path.join(t, "doc." + kind)
    if kind == "docx":
        docgen.write_docx(path, pw, seed)
        return [office2john.get_hash(path)]
    if kind == "odt":
        docgen.write_odt(path, pw, seed)
        return [odt2hashes.get_hashes(path, False)]
    docgen.write_pdf(path, pw, seed, **kw)
    return [pdf2john.get_hash(path)]


def _fields(stream):
    import contextlib
    import io
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


@pytest.mark.parametrize("cs,n", [(ALNUM, 7), (LOWER, 8), (ALNUM, 6)])
def test_deep_index_round_trip(cs, n):
    space = len(cs) ** n
    for i in (0, 1, 2 ** 32 - 1, 2 ** 32, 2 ** 32 + 12345, space // 3, space - 1):
        assert index_of(word(i, cs, n), cs) == i


@pytest.mark.parametrize("name,kind,kw,cs,pw,window", CASES, ids=[c[0] for c in CASES])
def test_planted_documents_verify_on_the_oracle(oracle, name, kind, kw, cs, pw, window):
    with tempfile.TemporaryDirectory() as t:
        for stream in _doc_streams(t, kind, kw, pw, 0xD9F):
            ctx = oracle.Ctx(stream)
            assert ctx.verify(pw.encode()) == 1, name
            assert ctx.verify(word(index_of(pw, cs) ^ 1, cs, len(pw)).encode()) == 0, name


@pytest.mark.gpu
@pytest.mark.parametrize("name,kind,kw,cs,pw,window", CASES, ids=[c[0] for c in CASES])
def test_planted_password_at_full_keyspace_positions(oracle, name, kind, kw, cs, pw, window):
    from dprf_amd import _lib
    n = len(pw)
    space = len(cs) ** n
    idx = index_of(pw, cs)
    start = max(0, min(idx - window // 2, space - window))
    count = min(window, space - start)
    assert start <= idx < start + count
    with tempfile.TemporaryDirectory() as t:
        for stream in _doc_streams(t, kind, kw, pw, 0xD9F):
            octx = oracle.Ctx(stream)
            with _lib.Context(_fields(stream), device=0) as ctx:
                hits, nh, st = ctx.search_range(cs, n, start, count)
                assert st["candidates"] == count and nh == len(hits), name
                assert idx in hits, (name, start, count, hits[:8])
                for h in hits:
                    assert octx.verify(word(h, cs, n).encode()) == 1, (name, h)
                # stop_on_first returns the lowest hit of the window
                fh, _, _ = ctx.search_range(cs, n, start, count, stop_on_first=True)
                assert fh and min(fh) == min(hits), name

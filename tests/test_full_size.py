"""BASELINE.json's configs at their full keyspace sizes, through position properties that do not need the
whole space scanned: a self-generated document (tests/docgen.py) whose password sits deep in the config's
keyspace -- past 2^32 for the alnum^7 and lowercase^8 spaces (the u64 enumeration of brute_force.py:199-219
and of the server's global order), or at its very last index -- is searched in range mode over a window
around that index at the config's own charset and length.  The lowest hit must be the planted index, and
every hit the GPU reports must verify on the oracle (the CPU restatement of the reference verifiers).

Two-way at full size (TWO_WAY): a complete sub-window deep in the config's keyspace is scanned by both, and
the GPU's hit set must EQUAL the oracle's: no false negative anywhere in the window, not only "the planted
index is found".  Windows follow the oracle's speed: >= 2^20 indices for PDF R2, R3/R4, R5, 2^17 for both
ODF streams (the `-e` stream's 2-byte check lets ~2^-16 false positives through), 2^14 for PDF R6 and 2^13
for Office (50,000 SHA-1 per candidate).  Past 2^32 wherever the config's keyspace reaches it (lowercase^6,
configs[3], has 3.1e8 indices: there the window sits in its upper half).
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
    # R6 at the other column shapes of range mode (dprf_kernels_r6.hip r6_pat_words): odd length (blocks at odd
    # offsets, the fifth word and a partial wrap) and a multiple of 4 (every block word-aligned, 20-word columns)
    ("pdf-r6-lower7", "pdf", {"R": 6, "length": 256}, LOWER, "qnbvcxz", 1 << 17),
    ("pdf-r6-lower8", "pdf", {"R": 6, "length": 256}, LOWER, "plokijuh", 1 << 17),
    ("pdf-r2-alnum7", "pdf", {"R": 2, "length": 40}, ALNUM, "Mo3kV9b", 1 << 26),
    ("pdf-r5-alnum7-first", "pdf", {"R": 5, "length": 256}, ALNUM, "aaaaaaa", 1 << 26),
]


# (config, writer kind, writer kwargs, charset, password, window): complete windows, oracle == GPU
TWO_WAY = [
    ("pdf-r2-alnum7", "pdf", {"R": 2, "length": 40}, ALNUM, "Mo3kV9b", 1 << 22),
    ("configs2-pdf-r4-alnum7", "pdf", {"R": 4, "length": 128}, ALNUM, "q7ZpL02", 1 << 20),
    ("configs2-pdf-r3-alnum7-last", "pdf", {"R": 3, "length": 128}, ALNUM, "9999999", 1 << 20),
    ("pdf-r5-alnum7-deep", "pdf", {"R": 5, "length": 256}, ALNUM, "Kq3Zr8w", 1 << 24),
    ("configs1-odt-e-alnum6", "odt_e", {}, ALNUM, "Zx9Qa7", 1 << 17),
    # the slow ones, on windows the oracle scans in seconds on the box's 16 CPUs
    ("configs0-office-pr8", "docx", {}, LOWER, "pwzqxkmv", 1 << 13),
    ("configs1-odt-alnum6", "odt", {}, ALNUM, "Zx9Qa7", 1 << 17),
    ("configs3-pdf-r6-lower6", "pdf", {"R": 6, "length": 256}, LOWER, "zyxwvu", 1 << 14),
    ("pdf-r6-lower7", "pdf", {"R": 6, "length": 256}, LOWER, "qnbvcxz", 1 << 12),
    ("pdf-r6-lower8", "pdf", {"R": 6, "length": 256}, LOWER, "plokijuh", 1 << 12),
]
ORACLE_THREADS = 16      # the GPU box's CPU share


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
    if kind in ("odt", "odt_e"):
        path = os.path.join(t, "doc.odt")
        docgen.write_odt(path, pw, seed)
        return [odt2hashes.get_hashes(path, kind == "odt_e")]
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


@pytest.mark.parametrize("name,kind,kw,cs,pw,window", CASES + TWO_WAY, ids=[c[0] for c in CASES + TWO_WAY])
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


def _window(pw, cs, window):
    n = len(pw)
    space = len(cs) ** n
    idx = index_of(pw, cs)
    start = max(0, min(idx - window // 2, space - window))
    return idx, start, min(window, space - start)


def test_two_way_windows_are_deep():
    for name, kind, kw, cs, pw, window in TWO_WAY:
        idx, start, count = _window(pw, cs, window)
        space = len(cs) ** len(pw)
        deep = 2 ** 32 if space > 2 ** 33 else space // 2
        assert start >= deep and count == window and start <= idx < start + count, name


@pytest.mark.gpu
@pytest.mark.parametrize("name,kind,kw,cs,pw,window", TWO_WAY, ids=[c[0] for c in TWO_WAY])
def test_full_window_hit_set_equals_oracle(oracle, name, kind, kw, cs, pw, window):
    """Both directions: every GPU hit is an oracle hit and every oracle hit is a GPU hit, over a complete
    window past 2^32 at the config's charset and length; and a two-device context on the one GPU agrees."""
    from dprf_amd import _lib
    n = len(pw)
    idx, start, count = _window(pw, cs, window)
    with tempfile.TemporaryDirectory() as t:
        for stream in _doc_streams(t, kind, kw, pw, 0xD9F):
            want, nwant = oracle.Ctx(stream).search_range(cs, n, start, count, nthreads=ORACLE_THREADS)
            assert idx in want, name
            for devs in ([0], [0, 0]):
                with _lib.Context(_fields(stream), devices=devs) as ctx:
                    hits, nh, st = ctx.search_range(cs, n, start, count)
                    assert st["candidates"] == count, (name, devs)
                    assert nh == nwant and hits == want, (name, devs, len(hits), len(want))
                    fh, _, _ = ctx.search_range(cs, n, start, count, stop_on_first=True, cap=1)
                    assert fh == want[:1], (name, devs)

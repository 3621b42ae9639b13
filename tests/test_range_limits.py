"""Range mode at the length limits, every format (round 5).  brute_force.py enumerates -pr N over lengths 1..N
(:199-219); the library spells a keyspace index on the device for any length up to DPRF_MAX_RANGE_LEN = 32 bytes.
Each case plants a password of length 1, 4, 5, 16, 17, 19, 20, 31 or 32 (every candidate-word boundary, Office's
one-to-two SHA-1 block edge after its 16-byte salt, PDF R2-R4's 32-byte truncation point, Office's 64-byte UTF-16 slot) in a
self-generated document (tests/docgen.py) and searches a window around its keyspace index over a two-character
charset (so 2^32 indices reach length 32), plus a 10-character alphanumeric one past 2^32.  The planted index must be
the lowest hit, every hit must verify on the oracle (the CPU restatement of the reference verifiers), and over a
sub-window around it the oracle scans in about a second the GPU's hit set must equal the oracle's."""
import contextlib
import io
import os
import tempfile

import pytest

AB = "ab"
ALNUM = "abcdefghijklmnopqrstuvwxyz" + "abcdefghijklmnopqrstuvwxyz".upper() + "0123456789"

# (format id, writer kind, writer kwargs, indices around the planted one the oracle also scans: sized to ~1 s of
# the oracle on the box's 16 CPUs; Office's 50,000 SHA-1 per candidate get the planted check only)
FORMATS = [
    ("office", "docx", {}, 0),
    ("odt", "odt", {}, 3000),
    ("pdf_r2", "pdf", {"R": 2, "length": 40}, 3000),
    ("pdf_r3", "pdf", {"R": 3, "length": 128}, 3000),
    ("pdf_r4", "pdf", {"R": 4, "length": 128}, 3000),
    ("pdf_r6", "pdf", {"R": 6, "length": 256}, 256),
    ("pdf_r5", "pdf", {"R": 5, "length": 256}, 3000),      # R5 range mode at the length limits too
]
PASSWORDS = [
    (AB, "b"),
    (AB, "abba"),
    (AB, "babab"),
    (AB, "ab" * 8),
    (AB, "ba" * 8 + "b"),
    (AB, "abbaabbaabbaabbaabb"),    # 19: Office's salt + UTF-16 = 54 bytes, one SHA-1 block
    (AB, "baabbaabbaabbaabbaab"),   # 20: 56 bytes, two blocks
    (AB, "a" + "ba" * 15),
    (AB, "b" * 31 + "a"),
    (ALNUM, "Zq7pLm0a9X"),
]
WINDOW = 3000


def index_of(pw, cs):
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


def _stream(t, kind, kw, pw):
    import docgen
    from dprf_amd.parsers import odt2hashes, office2john, pdf2john
    if kind == "docx":
        path = os.path.join(t, "d.docx")
        docgen.write_docx(path, pw, 0x1E7)
        return office2john.get_hash(path)
    if kind == "odt":
        path = os.path.join(t, "d.odt")
        docgen.write_odt(path, pw, 0x1E7)
        return odt2hashes.get_hashes(path, False)
    path = os.path.join(t, "d.pdf")
    docgen.write_pdf(path, pw, 0x1E7, **kw)
    return pdf2john.get_hash(path)


def _fields(stream):
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def _window(pw, cs, size=WINDOW):
    space = len(cs) ** len(pw)
    idx = index_of(pw, cs)
    start = max(0, min(idx - size // 2, space - size))
    return idx, start, min(size, space - start)


def test_cases_cover_the_length_limits():
    lens = {len(pw) for _, pw in PASSWORDS}
    assert {1, 4, 5, 16, 17, 19, 20, 31, 32} <= lens
    idx, start, count = _window(*reversed(PASSWORDS[-1]))
    assert start > 2 ** 32 and start <= idx < start + count


@pytest.mark.parametrize("fmt,kind,kw,two_way", FORMATS, ids=[f[0] for f in FORMATS])
def test_planted_length_limit_documents_verify_on_the_oracle(oracle, fmt, kind, kw, two_way):
    """the documents themselves: the planted password verifies on the oracle, its neighbour does not"""
    with tempfile.TemporaryDirectory() as t:
        for cs, pw in (PASSWORDS[0], PASSWORDS[-2]):
            octx = oracle.Ctx(_stream(t, kind, kw, pw))
            assert octx.verify(pw.encode()) == 1, (fmt, pw)
            other = word(index_of(pw, cs) ^ 1, cs, len(pw))
            assert octx.verify(other.encode()) == 0, (fmt, other)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,kind,kw,two_way", FORMATS, ids=[f[0] for f in FORMATS])
def test_range_mode_at_the_length_limits(oracle, fmt, kind, kw, two_way):
    from dprf_amd import _lib
    with tempfile.TemporaryDirectory() as t:
        for cs, pw in PASSWORDS:
            stream = _stream(t, kind, kw, pw)
            octx = oracle.Ctx(stream)
            n = len(pw)
            idx, start, count = _window(pw, cs)
            with _lib.Context(_fields(stream), device=0) as ctx:
                hits, nh, st = ctx.search_range(cs, n, start, count)
                assert st["candidates"] == count and nh == len(hits), (fmt, pw)
                assert hits and hits[0] == idx, (fmt, pw, start, count, hits[:4])
                for h in hits:
                    assert octx.verify(word(h, cs, n).encode()) == 1, (fmt, pw, h)
                if two_way:
                    _, s2, c2 = _window(pw, cs, two_way)
                    want, nwant = octx.search_range(cs, n, s2, c2, nthreads=16)
                    got, ngot, _ = ctx.search_range(cs, n, s2, c2)
                    assert got == want and ngot == nwant and idx in want, (fmt, pw, got[:4], want[:4])


# list mode: a password whose converted form fills the 64-byte slot exactly (Office 32 UTF-16 units, the rest 64
# bytes), with its 63- and 65-byte neighbours (65: the long sub-list) -- round 5 found the slot-filling case lost
# its SHA terminator in the Office and ODF kernels
SLOT_FORMATS = FORMATS


def _slot_password(fmt):
    if fmt == "office":
        return "Sl0tFi11ing-" + "x" * 19 + "é"            # 32 UTF-16 units = 64 bytes
    return "slot-filling:" + "0123456789abcdef" * 3 + "abc"     # 64 bytes


def test_slot_passwords_fill_the_slot():
    assert len(_slot_password("office").encode("utf-16-le")) == 64
    assert len(_slot_password("odt").encode()) == 64


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,kind,kw,two_way", SLOT_FORMATS, ids=[f[0] for f in SLOT_FORMATS])
def test_list_candidates_that_fill_the_slot(oracle, fmt, kind, kw, two_way):
    from dprf_amd import _lib
    pw = _slot_password(fmt)
    words = [pw[:-1], pw, pw + "z", pw[:-1] + "q", "z" + pw[1:], pw[:-1] + "q" + "z"]
    with tempfile.TemporaryDirectory() as t:
        stream = _stream(t, kind, kw, pw)
    want = [i for i, v in enumerate(oracle.Ctx(stream).verify_list(words)) if v == 1]
    assert 1 in want, fmt
    for devs in ([0], [0, 0]):
        with _lib.Context(_fields(stream), devices=devs) as ctx:
            hits, nh, st = ctx.verify_list(words)
            assert hits == want and st["candidates"] == len(words), (fmt, devs, hits, want)


# windows that cross 2^32: the library's launches carry a 64-bit start and 32-bit offsets within a launch, and its
# chunking cuts calls at launch sizes; a planted password just below and just above 2^32
CROSS = [("pdf_r5", "pdf", {"R": 5, "length": 256}), ("pdf_r4", "pdf", {"R": 4, "length": 128}),
         ("odt", "odt", {})]


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,kind,kw", CROSS, ids=[c[0] for c in CROSS])
def test_windows_across_2_32(oracle, fmt, kind, kw):
    from dprf_amd import _lib
    n = 7
    for idx in (2 ** 32 - 1, 2 ** 32):
        pw = word(idx, ALNUM, n)
        with tempfile.TemporaryDirectory() as t:
            stream = _stream(t, kind, kw, pw)
        assert oracle.Ctx(stream).verify(pw.encode()) == 1
        with _lib.Context(_fields(stream), devices=[0, 0]) as ctx:
            for start, count in ((2 ** 32 - 1500, 3000), (idx, 1), (2 ** 32 - 2 ** 21, 2 ** 22)):
                hits, _, st = ctx.search_range(ALNUM, n, start, count)
                assert st["candidates"] == count and hits == [idx], (fmt, idx, start, count, hits)

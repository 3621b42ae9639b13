"""PDF R5 range mode by runs (round 5, dprf_kernels.hip k_pdf_r5 R5_RUNS): each thread verifies a run of PER
consecutive keyspace indices (PER 16 for charsets of 16 or more characters, 8 for 8-15), spelled from two full
spellings (the run's first index, and the first index past the one wrap of the last digit) plus one charset byte
per candidate, with one kernel instantiation per number of candidate words (pwlen 1-4 / 5-8 / 9-12 / 13-16 / longer).  These tests plant a password and search windows that
put it at every position of a run (before and after the wrap of the last digit), at the ragged end of a launch and
outside the window, for every word-count class, every byte position of the last character, charsets of exactly
16 and 8 characters and ones smaller than 8 (the per-candidate path), against the oracle (the CPU restatement
of pdf_password_verifier.c:194-221).  The reference verdicts of R5 documents are pinned separately
(tests/golden, test_gpu_parity.py)."""
import os
import tempfile

import pytest

LOWER = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWER + LOWER.upper() + "0123456789"


def per(cs):
    """the run length k_pdf_r5 takes for this charset (launch_pdf_r5); < 8 characters: no runs"""
    return 16 if len(cs) >= 16 else 8


# (charset, password): the last character sits right after the wrap of the last digit (a low digit), so runs
# that start up to PER - 1 indices earlier cross the wrap
CASES = [
    (ALNUM, "Kq3Zr8b"),             # configs' shape: 7 chars, 2 candidate words, last char in byte 2
    (LOWER, "qc"),                  # 1 word, byte 1
    (LOWER, "zyxa"),                # 1 word, byte 3
    (ALNUM, "Mo3kV9bc"),            # 2 words, byte 3
    (LOWER, "passwordb"),           # 3 words, byte 0
    ("abcdefgh", "hgfedcbahgfeb"),  # 4 words (13 chars), byte 0; cslen 8: runs of 8
    ("0123456789abcdef", "c0ffee5"),  # cslen 16: runs of 16 through the wrap
    ("0123456789", "20241231"),     # digits: runs of 8
    ("ab", "abbabaabbabaabbabab"),  # 19 chars: the generic instantiation; cslen < 8: per-candidate path
    # 17-32 characters on the RUN path (the 8-word instantiation with runs had no case)
    ("0123456789", "31415926535897932"),              # 17 chars, runs of 8, byte 0 of word 4
    ("0123456789abcdef", "0" * 20 + "deadbeefca1"),   # 31 chars, runs of 16, byte 2 of word 7
    ("abcdefgh", "a" * 28 + "hgcb"),                  # 32 chars: the last slot byte, runs of 8
    ("0123456", "6543210"),         # cslen 7: per-candidate path
]


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


def _stream(t, pw):
    import docgen
    from dprf_amd.parsers import pdf2john
    path = os.path.join(t, "r5.pdf")
    docgen.write_pdf(path, pw, 0x5A5, R=5, length=256)
    return pdf2john.get_hash(path)


def _fields(stream):
    import contextlib
    import io
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def windows(idx, space, run):
    """(start, count) windows around idx: idx at every run position r < run, past a first run, and in later blocks, with
    the window ending 1 / 5 / 300 past it (a ragged last run and block), and two windows that miss it."""
    out = []
    for r in list(range(run)) + [run + 3, 4096 + 5, 8192 + 4095]:
        for tail in (1, 5, 300):
            start = idx - r
            if start < 0 or start + r + tail > space:
                continue
            out.append((start, r + tail, True))
    if idx >= 50:
        out.append((idx - 50, 50, False))
    if idx + 1 + 40 <= space:
        out.append((idx + 1, 40, False))
    return out


def test_cases_cover_the_run_shapes():
    for cs, pw in CASES:
        assert index_of(word(index_of(pw, cs), cs, len(pw)), cs) == index_of(pw, cs)
        assert len(cs) < 8 or cs.index(pw[-1]) < per(cs) - 1      # runs through it cross the wrap
    nw = {(len(pw) + 3) // 4 if len(pw) <= 16 else 8 for _, pw in CASES}
    assert nw == {1, 2, 3, 4, 8}
    assert {(len(pw) - 1) % 4 for _, pw in CASES} == {0, 1, 2, 3}
    assert {len(cs) for cs, _ in CASES} >= {7, 8, 10, 16, 26, 62}
    assert {len(pw) for cs, pw in CASES if len(cs) >= 8 and len(pw) > 16} == {17, 31, 32}


@pytest.mark.parametrize("cs,pw", CASES, ids=[pw for _, pw in CASES])
def test_planted_r5_documents_verify_on_the_oracle(oracle, cs, pw):
    with tempfile.TemporaryDirectory() as t:
        octx = oracle.Ctx(_stream(t, pw))
        assert octx.verify(pw.encode()) == 1
        idx = index_of(pw, cs)
        for j in (idx - 1, idx + 1):
            if 0 <= j < len(cs) ** len(pw):
                assert octx.verify(word(j, cs, len(pw)).encode()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("cs,pw", CASES, ids=[pw for _, pw in CASES])
def test_r5_runs_find_the_password_at_every_run_position(cs, pw):
    from dprf_amd import _lib
    n = len(pw)
    idx = index_of(pw, cs)
    space = len(cs) ** n
    with tempfile.TemporaryDirectory() as t:
        fields = _fields(_stream(t, pw))
    with _lib.Context(fields, device=0) as ctx:
        for start, count, inside in windows(idx, space, per(cs)):
            hits, nh, st = ctx.search_range(cs, n, start, count)
            assert st["candidates"] == count, (pw, start, count)
            assert hits == ([idx] if inside else []) and nh == len(hits), (pw, start, count, hits)
            if inside:
                fh, _, _ = ctx.search_range(cs, n, start, count, stop_on_first=True, cap=1)
                assert fh == [idx], (pw, start, count)
    # two device lanes on the one GPU: the call is cut into chunks, each launch's runs start at its own chunk start
    with _lib.Context(fields, devices=[0, 0]) as ctx:
        big = max(0, min(idx - (1 << 23) - 3, space - (1 << 24)))         # 2^24 indices: chunks on both lanes
        for start, count, inside in windows(idx, space, per(cs))[-8:] + [(big, min(1 << 24, space - big), True)]:
            hits, _, st = ctx.search_range(cs, n, start, count)
            assert st["candidates"] == count and hits == ([idx] if inside else []), (pw, start, count, hits)

"""PDF R5 list launches by candidate length (round 6): launch_pdf_r5 runs a list launch whose longest candidate has at
most 8 / 16 bytes through k_pdf_r5<1, 2, 8> / <1, 4, 8> (one message block: the password words, the 8 salt bytes and
0x80 in the first NW + 3 words, the round-61 early exit), longer ones through <1, 8, 8> (the two-block path).  Every
verdict must equal the oracle's (the CPU restatement of pdf_password_verifier.c:194-221) whatever path the launch
takes, at every length at and around the path edges, with the planted password found on each path; device-spelled
symbol windows (whose longest candidate bounds the path) land on the short paths too."""
import contextlib
import io
import os
import random
import tempfile

import pytest

LENGTHS = [0, 1, 3, 4, 5, 7, 8, 9, 12, 15, 16, 17, 23, 31, 32, 33, 40, 47]


def _doc(pw, seed=0x7A5):
    import docgen
    from dprf_amd.parsers import pdf2john
    with tempfile.TemporaryDirectory() as t:
        p = os.path.join(t, "d.pdf")
        docgen.write_pdf(p, pw, seed, R=5, length=256)
        return pdf2john.get_hash(p)


def _fields(stream):
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def _lists(pw, cap):
    """random candidates of at most `cap` bytes (every length up to it present) with the password planted twice"""
    rng = random.Random(cap * 31 + len(pw))
    al = "abcdefghijklmnopqrstuvwxyz0123456789"
    words = ["".join(rng.choice(al) for _ in range(n)) for n in range(cap + 1) for _ in range(3)]
    words += [pw[:-1] + "Z" if pw else "Z", pw + "a"][: 2 if len(pw) < cap else 1]
    k = rng.randrange(len(words))
    words[k:k] = [pw]
    words.append(pw)
    return words


@pytest.mark.parametrize("pwlen", [0, 6, 8, 13, 16])
def test_lists_verify_on_the_oracle(oracle, pwlen):
    pw = "pw5" * 6
    pw = pw[:pwlen]
    c = oracle.Ctx(_doc(pw))
    for cap in (8, 16, 47):
        if pwlen > cap:
            continue
        words = _lists(pw, cap)
        v = c.verify_list([w.encode() for w in words])
        assert [i for i, x in enumerate(v) if x == 1] == [i for i, w in enumerate(words) if w == pw]


@pytest.mark.gpu
@pytest.mark.parametrize("pwlen", [0, 6, 8, 13, 16])
def test_gpu_list_paths_by_length(oracle, pwlen):
    from dprf_amd import _lib
    pw = ("pw5" * 6)[:pwlen]
    stream = _doc(pw)
    c = oracle.Ctx(stream)
    with _lib.Context(_fields(stream), device=0) as ctx:
        for cap in (8, 16, 47):                           # the <1,2,8>, <1,4,8> and <1,8,8> launches
            if pwlen > cap:
                continue
            words = _lists(pw, cap)
            expect = [i for i, x in enumerate(c.verify_list([w.encode() for w in words])) if x == 1]
            hits, _, _ = ctx.verify_list(words)
            assert hits == expect and expect, (pwlen, cap, hits, expect)


@pytest.mark.gpu
def test_gpu_list_every_length_at_the_path_edges(oracle):
    """one list per length: a launch of candidates all of exactly that length (the path is chosen by the launch's
    longest), 600 random candidates each, verdicts against the oracle"""
    from dprf_amd import _lib
    stream = _doc("x")
    c = oracle.Ctx(stream)
    rng = random.Random(5)
    with _lib.Context(_fields(stream), device=0) as ctx:
        for n in LENGTHS:
            words = ["".join(rng.choice("xyz") for _ in range(n)) for _ in range(600)]
            expect = [i for i, x in enumerate(c.verify_list([w.encode() for w in words])) if x == 1]
            hits, _, _ = ctx.verify_list(words)
            assert hits == expect, (n, hits[:5], expect[:5])
            if n == 1:
                assert expect                              # "x" itself is among them


@pytest.mark.gpu
def test_gpu_symbol_windows_on_the_short_paths():
    from dprf_amd import _lib
    stream = _doc("ωaω")
    with _lib.Context(_fields(stream), device=0) as ctx:
        for cs, n in (("aω", 3), ("aωé€", 3), ("a\U0001D11Eω", 5)):    # longest 6, 9, 20 bytes: all three paths
            hits, _, _ = ctx.search_symbols(cs, n, 0, len(cs) ** n)
            pw = "ωaω"
            want = [sum(cs.index(ch) * len(cs) ** (n - 1 - k) for k, ch in enumerate(pw))] if n == 3 else []
            assert hits == want, (cs, hits, want)

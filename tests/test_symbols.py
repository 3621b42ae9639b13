"""Range mode over multi-byte symbols spelled on the device (round 6, ABI 7: include/dprf.h dprf_search_symbols,
k_spell_symbols).  A --charset with non-ASCII characters enumerates its CHARACTERS in itertools.product order
(brute_force.py:205 over symbols); the device spells each candidate into a list slot and the list kernels verify it.

Parity: for every format, the hit set of a whole symbol window equals the hit set of the same window spelled on the
host (payload.spell_utf8) and verified in list mode, and the planted password is the oracle's (tests/docgen.py writes
the documents, pyoracle is the CPU restatement of the reference verifiers).  The symbols cover 1- to 4-byte UTF-8
characters (Office: BMP and a surrogate pair in UTF-16LE), PDF R2-R4's truncation at 32 bytes, windows over several
chunks on two streams (R2-R4) and two device lanes, and the slot limit (E_PWLEN, brute_force then spells on the
host)."""
import contextlib
import io
import os
import tempfile

import pytest

SYMS = "aé€\U0001D11Eb"          # 1, 2, 3, 4, 1 UTF-8 bytes
PW = "é\U0001D11Ea"


def _doc(kind, kw, pw, seed=0x5E1):
    import docgen
    from dprf_amd.parsers import odt2hashes, office2john, pdf2john
    with tempfile.TemporaryDirectory() as t:
        if kind == "docx":
            p = os.path.join(t, "d.docx")
            docgen.write_docx(p, pw, seed)
            return office2john.get_hash(p)
        if kind == "odt":
            p = os.path.join(t, "d.odt")
            docgen.write_odt(p, pw, seed)
            return odt2hashes.get_hashes(p, False)
        p = os.path.join(t, "d.pdf")
        docgen.write_pdf(p, pw, seed, **kw)
        return pdf2john.get_hash(p)


def _fields(stream):
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def _index(cs, pw):
    i = 0
    for ch in pw:
        i = i * len(cs) + cs.index(ch)
    return i


KINDS = [("docx", {}), ("odt", {}), ("pdf", {"R": 2, "length": 40}), ("pdf", {"R": 4, "length": 128}),
         ("pdf", {"R": 5, "length": 256}), ("pdf", {"R": 6, "length": 256})]
IDS = ["office", "odt", "pdf-r2", "pdf-r4", "pdf-r5", "pdf-r6"]


@pytest.mark.parametrize("kind,kw", KINDS, ids=IDS)
def test_planted_documents_verify_on_the_oracle(oracle, kind, kw):
    c = oracle.Ctx(_doc(kind, kw, PW))
    assert c.verify(PW.encode()) == 1 and c.verify("éa\U0001D11E".encode()) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", KINDS, ids=IDS)
def test_device_spelled_window_equals_host_spelled_list(kind, kw):
    from dprf_amd import _lib
    from dprf_amd.payload import spell_utf8
    stream = _doc(kind, kw, PW)
    n = len(SYMS) ** 3
    blob, offs = spell_utf8(SYMS, 3, 0, n)
    for devs in ([0], [0, 0]):
        with _lib.Context(_fields(stream), devices=devs) as ctx:
            hs, nh, st = ctx.search_symbols(SYMS, 3, 0, n)
            hl, _, _ = ctx.verify_blob(blob, offs)
            assert hs == hl == [_index(SYMS, PW)], (kind, devs, hs, hl)
            assert st["candidates"] == n
            # a window that starts inside the keyspace: indices stay keyspace indices
            hs2, _, _ = ctx.search_symbols(SYMS, 3, 7, n - 7, stop_on_first=True)
            assert hs2 == [_index(SYMS, PW)]


@pytest.mark.gpu
def test_pdf_r4_truncates_symbol_candidates_at_32_bytes():
    """R2-R4 hash the first 32 bytes of the password (pdf...c:137): 17 two-byte characters are 34 bytes, so every
    candidate that shares the planted password's first 16 characters verifies -- the same set list mode finds."""
    from dprf_amd import _lib
    from dprf_amd.payload import spell_utf8
    greek = "αβγδεζηθ"
    pw = "βγ" * 8 + "δ"
    stream = _doc("pdf", {"R": 4, "length": 128}, pw)
    base = _index(greek, pw) - greek.index("δ")            # the 8 variants of the 17th character
    s, n = base - 100, 300
    blob, offs = spell_utf8(greek, 17, s, n)
    with _lib.Context(_fields(stream), device=0) as ctx:
        hs, _, _ = ctx.search_symbols(greek, 17, s, n)
        hl, _, _ = ctx.verify_blob(blob, offs)
    assert hs == [base + k for k in range(8)] == [s + h for h in hl]


@pytest.mark.gpu
def test_window_over_several_chunks_and_streams():
    """A 2^25 + 2^20 window of 2-byte symbols on PDF R4 (launches of up to 2^24 alternate two streams, each with its
    own spelled-slot buffer) and on two device lanes: the one planted hit near the end, and stop_on_first's lowest."""
    from dprf_amd import _lib
    greek = "αβγδεζηθικλμνξοπρστυφχψω"                      # 24 symbols
    pw = "ωψχφυτ"
    stream = _doc("pdf", {"R": 4, "length": 128}, pw)
    idx = _index(greek, pw)
    n = (1 << 25) + (1 << 20)
    s = idx - n + 12345
    for devs in ([0], [0, 0]):
        with _lib.Context(_fields(stream), devices=devs) as ctx:
            hs, _, st = ctx.search_symbols(greek, 6, s, n)
            assert hs == [idx] and st["candidates"] == n, (devs, hs, st)
            assert st["launches"] >= 2
            hs, _, _ = ctx.search_symbols(greek, 6, s, n, stop_on_first=True)
            assert hs == [idx]


@pytest.mark.gpu
def test_candidates_over_a_slot_are_refused_and_brute_force_spells_them_on_the_host():
    from dprf_amd import _lib, brute_force as bf
    pw = "\U0001D11E" * 17                                # 68 UTF-8 bytes: over a 64-byte slot
    stream = _doc("odt", {}, pw)
    with _lib.Context(_fields(stream), device=0) as ctx:
        with pytest.raises(_lib.DprfError) as ei:
            ctx.search_symbols("\U0001D11Ea", 17, 0, 16)
        assert ei.value.code == _lib.E_PWLEN
        found, _ = bf.search_round(ctx, "a\U0001D11E", 17, (1 << 17) - 4, 4)
        assert found == (1 << 17) - 1                     # the last index: every position the second symbol


@pytest.mark.gpu
def test_bad_symbol_tables_are_refused():
    """DPRF_E_CHARSET before any device work: empty, repeated, NUL-carrying or over-4-byte symbols; for Office a symbol
    that is not one valid UTF-8 character (its UTF-16LE would be undefined, msoffcrypto...c:287-336)."""
    import ctypes
    from dprf_amd import _lib
    L = _lib.lib()

    def call(ctx, syms, pwlen=2):
        offs = [0]
        for b in syms:
            offs.append(offs[-1] + len(b))
        nh = ctypes.c_int64()
        hits = (ctypes.c_uint64 * 1)()
        return L.dprf_search_symbols(ctx._h, b"".join(syms), (ctypes.c_uint32 * len(offs))(*offs), len(syms), pwlen,
                                     0, 4, 0, hits, 1, ctypes.byref(nh), None)
    with _lib.Context(_fields(_doc("pdf", {"R": 4, "length": 128}, PW)), device=0) as ctx:
        for bad in ([b"a", b""], [b"a", b"a"], [b"a\x00"], [b"abcde"], []):
            assert call(ctx, bad) == _lib.E_CHARSET, bad
        assert call(ctx, [b"\xc3", b"\xa9"]) == 0           # PDF: raw byte symbols are symbols
        assert call(ctx, [b"a", b"b"], pwlen=33) == _lib.E_PWLEN
    with _lib.Context(_fields(_doc("docx", {}, PW)), device=0) as ctx:
        for bad in ([b"\xc3"], [b"ab"], [b"\xed\xa0\x80"]):  # truncated, two characters, a lone surrogate
            assert call(ctx, bad) == _lib.E_CHARSET, bad
        assert call(ctx, ["é".encode(), "\U0001D11E".encode()]) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", [("odt", {}), ("docx", {}), ("pdf", {"R": 6, "length": 256}),
                                     ("pdf", {"R": 5, "length": 256})], ids=["odt", "office", "pdf-r6", "pdf-r5"])
def test_slot_filling_symbol_candidates(kind, kw):
    """Candidates of up to exactly 64 bytes (16 four-byte characters: the SHA terminator falls in the word after the
    slot, the round-5 slot-edge bug class) and 60 bytes, spelled on the device: the planted password found at its
    index, the same hits as the host-spelled list."""
    from dprf_amd import _lib
    from dprf_amd.payload import spell_utf8
    cs = "a\U0001D11E"
    for n in (16, 15):
        pw = "\U0001D11E" * n                                  # 4n bytes of UTF-8 (Office: 4n of UTF-16LE)
        stream = _doc(kind, kw, pw)
        idx = (1 << n) - 1
        s, cnt = (1 << n) - 64, 64
        blob, offs = spell_utf8(cs, n, s, cnt)
        with _lib.Context(_fields(stream), device=0) as ctx:
            hs, _, _ = ctx.search_symbols(cs, n, s, cnt)
            hl, _, _ = ctx.verify_blob(blob, offs)
        assert hs == [idx] == [s + h for h in hl], (kind, n, hs, hl)

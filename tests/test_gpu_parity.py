"""GPU parity: libdprf.so's kernels vs the reference's verdicts (golden fixtures) and vs the oracle, through
the C ABI.  Bit-exact: hit sets must be identical."""
import os
import random
import tempfile
import zlib

import pytest

pytestmark = pytest.mark.gpu

LOWER = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWER + LOWER.upper() + "0123456789"


@pytest.fixture(scope="module")
def dprf():
    from dprf_amd import _lib
    assert _lib.device_count() >= 1, "no gfx950 device: GPU tests need the MI355X box"
    return _lib


def ctx_for(dprf, streams, name):
    from dprf_amd import brute_force as bf
    return dprf.Context(bf.parse_verification_data(streams[name]["stream"]))


def test_kernel_families(dprf, streams):
    want = {"office": "office_std", "odt": "odf_aes256"}
    for name in streams:
        c = ctx_for(dprf, streams, name)
        fam = c.kernel
        if name.startswith("pdf"):
            assert fam.startswith("pdf_r"), (name, fam)
        else:
            assert fam == want[name.split("_")[0]], (name, fam)


def test_verdict_tables_match_reference(dprf, streams, verdicts):
    for name, table in verdicts.items():
        c = ctx_for(dprf, streams, name)
        cands = [p for p, _ in table]
        hits, n, st = c.verify_list(cands)
        want = [i for i, (_, v) in enumerate(table) if v]
        assert hits == want, (name, [cands[i] for i in hits], [cands[i] for i in want])
        assert st["candidates"] == len(cands)


def _long_ctx(dprf, d, devices=None):
    from dprf_amd import brute_force as bf
    return dprf.Context(bf.parse_verification_data(d["stream"]), devices=devices)


def test_long_candidates_match_reference(dprf, long_verdicts):
    """Round 4: candidates of 64/65/119/120/127/128/176 bytes and multi-byte UTF-8 (2-, 3-, 4-byte
    sequences) on documents whose passwords are long themselves (tests/golden/make_long.py): the GPU's hits equal the
    reference executables' exit codes, short and long candidates mixed in one list.  R6 candidates over 176 bytes,
    where the reference aborts (-6) or crashes (-11), are DPRF_E_DOMAIN -- in the status call and when verified."""
    for name, d in long_verdicts.items():
        ok = [(p, v) for p, v in d["verdicts"] if v in (0, 1)]
        bad = [p for p, v in d["verdicts"] if v not in (0, 1)]
        c = _long_ctx(dprf, d)
        hits, n, st = c.verify_list([p for p, _ in ok])
        want = [i for i, (_, v) in enumerate(ok) if v]
        assert hits == want and n == len(want), (name, [ok[i][0] for i in hits], [ok[i][0] for i in want])
        assert st["candidates"] == len(ok)
        assert any(len(p.encode()) > 64 for p, _ in ok), name
        if bad:
            from dprf_amd import payload as pl
            blob, offs = pl._pack(bad)
            assert [int(v) for v in c.list_status(blob, offs)] == [dprf.E_DOMAIN] * len(bad), name
            with pytest.raises(dprf.DprfError) as ei:
                c.verify_list(bad[:1])
            assert ei.value.code == dprf.E_DOMAIN
        c.close()


def test_long_and_short_lowest_hit_across_sub_lists(dprf, long_verdicts):
    """stop_on_first over a list mixing slot-sized and long candidates: the answer is the lowest list index that
    verifies, whichever sub-list (slots or long records) holds it; list indices survive the split; two device lanes
    give the same answer."""
    d = long_verdicts["pdf_r5_long127"]
    pw = d["password"]
    rng = random.Random(3)
    words = ["".join(rng.choice(ALNUM) for _ in range(rng.choice((5, 40, 70, 100, 130)))) for _ in range(3000)]
    plant = {1717: pw + "-beyond-127-is-ignored", 2400: pw}
    for k, v in plant.items():
        words[k] = v
    for devs in ([0], [0, 0]):
        c = _long_ctx(dprf, d, devs)
        hits, n, st = c.verify_list(words)
        assert hits == sorted(plant) and n == 2 and st["candidates"] == len(words)
        h1, _, _ = c.verify_list(words, stop_on_first=True, cap=1)
        assert h1 == [1717]
        c.close()


def test_short_and_long_hits_on_one_document_stop_on_first(dprf, oracle):
    """a list whose hits sit in BOTH sub-lists of one document -- the ODF -e stream of odt_long_e_200 (its
    2-byte check, odt...c:98-101, accepts ~2^-16 of all candidates): the 200-byte password is a long hit and
    tests/golden/make_mixed.py found short candidates the reference verifier also accepts (exit code 1).  Under
    stop_on_first with cap = 1 the answer is the lowest LIST index whichever sub-list holds it: a short hit below a
    long one (the long sub-list is then cut to the records below it, dprf_host.cpp dprf_verify_list) and a long hit
    below a short one; on one device lane and on two.  The fillers are checked with the CPU oracle (a filler the -e
    check happened to accept would be a hit of its own)."""
    import json
    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "mixed_verdicts.json")))
    octx = oracle.Ctx(d["stream"])
    rng = random.Random(11)
    words = []
    while len(words) < 1500:
        w = "".join(rng.choice(ALNUM) for _ in range(rng.choice((6, 9, 70, 90))))
        if octx.verify(w) == 0:
            words.append(w)
    short, long_ = d["short_hits"][0], d["long_hit"]
    for plant in ({300: short, 900: long_}, {300: long_, 900: short}, {300: short, 301: short[::-1], 900: long_}):
        ws = list(words)
        for k, v in plant.items():
            ws[k] = v
        want = sorted(k for k, v in plant.items() if octx.verify(v) == 1)
        for devs in ([0], [0, 0]):
            c = _long_ctx(dprf, d, devs)
            hits, n, st = c.verify_list(ws)
            assert hits == want and n == len(want), (plant, devs, hits)
            h1, n1, st1 = c.verify_list(ws, stop_on_first=True, cap=1)
            assert h1 == [300], (plant, devs, h1)
            if plant[300] == short:    # the long records above the short hit are not verified at all
                assert st1["candidates"] <= len(ws) - sum(1 for w in ws[300:] if len(w.encode()) > 64), (devs, st1)
            c.close()


def test_long_list_over_several_launches(dprf, oracle, long_verdicts):
    """A long sub-list of 2^20 + 3 records (more than one long-list launch, LONG_HI = 2^20): 130-byte R5 candidates,
    which the reference truncates to 127 (pdf...c:197-200), with the 127-byte password as the prefix of four of them
    planted across the launch seam, and a near miss (last kept byte changed)."""
    import numpy as np
    d = long_verdicts["pdf_r5_long127"]
    pw = np.frombuffer(d["password"].encode(), dtype=np.uint8)
    n = (1 << 20) + 3
    blob = np.random.default_rng(5).integers(65, 91, size=(n, 130), dtype=np.uint8)
    plant = [0, (1 << 20) - 1, 1 << 20, n - 1]
    for k in plant + [7]:
        blob[k, :127] = pw
    blob[7, 126] ^= 1
    offs = np.arange(n + 1, dtype=np.uint64) * 130
    c = _long_ctx(dprf, d)
    hits, nh, st = c.verify_blob(blob.tobytes(), offs)
    assert hits == plant and nh == len(plant) and st["candidates"] == n and st["launches"] >= 2
    assert oracle.Ctx(d["stream"]).verify(bytes(blob[7])) == 0 and oracle.Ctx(d["stream"]).verify(bytes(blob[0])) == 1
    c.close()


def test_hitsets_match_reference(dprf, streams, hitsets):
    for key, h in hitsets.items():
        c = ctx_for(dprf, streams, h["stream"])
        hits, n, st = c.search_range(h["charset"], h["pwlen"], h["start"], h["count"])
        assert hits == h["hits"] and n == len(h["hits"]), key
        assert st["candidates"] == h["count"], key


def test_every_stream_finds_its_password_in_range_mode(dprf, streams):
    for name, d in streams.items():
        pw = d["password"]
        if len(pw) > 4 or any(ch not in ALNUM for ch in pw):
            continue
        cs = LOWER if all(ch in LOWER for ch in pw) else ALNUM
        idx = 0
        for ch in pw:
            idx = idx * len(cs) + cs.index(ch)
        c = ctx_for(dprf, streams, name)
        lo = max(0, idx - 3000)
        hits, n, _ = c.search_range(cs, len(pw), lo, min(6000, len(cs) ** len(pw) - lo))
        assert idx in hits, name


def _random_words(rng, n, lo=1, hi=12, alphabet=ALNUM):
    return ["".join(rng.choice(alphabet) for _ in range(rng.randint(lo, hi))) for _ in range(n)]


@pytest.mark.parametrize("name,n", [("pdf_testdoc_r2", 3000), ("pdf_testdoc_r4", 3000), ("pdf_synth_r3_l40_cab", 3000),
                                    ("pdf_synth_r4_meta0_dog", 3000), ("pdf_synth_r5_cat", 3000),
                                    ("pdf_synth_r6_ox", 150), ("odt_testdoc_e", 800), ("odt_testdoc_std", 400),
                                    ("office_testdoc", 24)])
def test_random_lists_vs_oracle(dprf, oracle, streams, name, n):
    rng = random.Random(zlib.crc32(name.encode()))      # str hash() is salted per process
    words = _random_words(rng, n) + [streams[name]["password"]]
    rng.shuffle(words)
    want = [i for i, v in enumerate(oracle.Ctx(streams[name]["stream"]).verify_list(words)) if v == 1]
    hits, _, _ = ctx_for(dprf, streams, name).verify_list(words)
    assert hits == want


# (writer kind, writer kwargs, candidates per document): every revision / key length / metadata flag the
# reference's verifiers accept (pdf_password_verifier.c:89-101), both ODF streams, Office
RANDOM_DOCS = [
    ("pdf", {"R": 2, "length": 40}, 2000), ("pdf", {"R": 3, "length": 128}, 2000),
    ("pdf", {"R": 3, "length": 40}, 2000), ("pdf", {"R": 4, "length": 128, "meta": False}, 2000),
    ("pdf", {"R": 4, "length": 128, "P": -4}, 2000), ("pdf", {"R": 5, "length": 256}, 2000),
    ("pdf", {"R": 6, "length": 256}, 120), ("odt", {}, 300), ("odt_e", {}, 600), ("docx", {}, 12),
]


def _near_misses(pw):
    """Candidates one edit away from the password (and the password itself)."""
    flip = chr(ord(pw[-1]) ^ 1)
    return [pw, pw[:-1], pw + "a", pw[:-1] + flip, pw.upper() if pw != pw.upper() else pw.lower(), "x" + pw]


@pytest.mark.parametrize("seed", [101, 202, 303])
@pytest.mark.parametrize("kind,kw,n", RANDOM_DOCS, ids=["%s%s" % (k, "".join("-%s%s" % i for i in sorted(w.items())))
                                                       for k, w, _ in RANDOM_DOCS])
def test_random_documents_vs_oracle(dprf, oracle, kind, kw, n, seed):
    """Fresh documents (tests/docgen.py: random salts, IVs, IDs, O values and passwords for each seed) through
    the parsers, then a random candidate list with the password and its near misses: GPU hit set == oracle's."""
    from test_full_size import _doc_streams, _fields
    rng = random.Random(seed * 1000 + zlib.crc32(repr((kind, sorted(kw.items()))).encode()))
    pw = "".join(rng.choice(ALNUM) for _ in range(rng.randint(3, 9)))
    with tempfile.TemporaryDirectory() as t:
        stream = _doc_streams(t, kind, kw, pw, seed)[0]
    words = _random_words(rng, n) + _near_misses(pw)
    rng.shuffle(words)
    want = [i for i, v in enumerate(oracle.Ctx(stream).verify_list(words)) if v == 1]
    assert words.index(pw) in want
    hits, _, st = dprf.Context(_fields(stream)).verify_list(words)
    assert hits == want
    assert st["candidates"] == len(words)


@pytest.mark.parametrize("name", ["pdf_synth_r2_key", "pdf_synth_r3_l128_abc", "pdf_synth_r5_cat", "pdf_synth_r6_ox",
                                  "odt_synth_std_zq", "office_synth_ok"])
def test_ragged_lengths_and_limits(dprf, oracle, streams, name):
    """Lengths 0..64 in one payload (32/33 around the PDF truncation, 55/56 around the SHA block edge)."""
    rng = random.Random(11)
    lens = list(range(0, 65)) if not name.startswith("office") else [1, 2, 19, 20, 27, 28, 31, 32]
    words = ["".join(rng.choice(ALNUM) for _ in range(k)) for k in lens] + [streams[name]["password"]]
    if name.startswith("office"):
        words = [w for w in words if w]
    want = [i for i, v in enumerate(oracle.Ctx(streams[name]["stream"]).verify_list(words)) if v == 1]
    hits, _, st = ctx_for(dprf, streams, name).verify_list(words)
    assert hits == want
    assert st["candidates"] == len(words)


def test_pdf_truncates_long_candidates_like_reference(dprf, oracle, streams):
    """R<=4 only looks at the first 32 bytes (pdf_password_verifier.c:137): candidates sharing a 32-byte
    prefix get the same verdict."""
    words = ["Q" * 32, "Q" * 33, "Q" * 40, "Q" * 64, "Q" * 31]
    want = [v for v in oracle.Ctx(streams["pdf_testdoc_r4"]["stream"]).verify_list(words)]
    hits, _, _ = ctx_for(dprf, streams, "pdf_testdoc_r4").verify_list(words)
    assert hits == [i for i, v in enumerate(want) if v == 1]


def test_office_utf8_candidates(dprf, oracle, streams):
    words = ["été", "passwörd", "ok", "日本語", "😀ok", "o", "k"]
    want = [i for i, v in enumerate(oracle.Ctx(streams["office_synth_ok"]["stream"]).verify_list(words)) if v == 1]
    hits, _, _ = ctx_for(dprf, streams, "office_synth_ok").verify_list(words)
    assert hits == want == [2]


def test_errors_are_errors_not_hits(dprf, streams):
    c = ctx_for(dprf, streams, "office_synth_ok")
    with pytest.raises(dprf.DprfError) as ei:
        c.verify_list([""])
    assert ei.value.code == dprf.E_DOMAIN
    with pytest.raises(dprf.DprfError) as ei:
        c.verify_list([b"\xff\xfe"])
    assert ei.value.code == dprf.E_DOMAIN
    with pytest.raises(dprf.DprfError) as ei:
        c.search_range("aé", 2, 0, 4)
    assert ei.value.code == dprf.E_CHARSET
    c2 = ctx_for(dprf, streams, "pdf_synth_r6_ox")
    c2.verify_list(["x" * 65, "y" * 176])                    # long candidates are verified (round 4)
    with pytest.raises(dprf.DprfError) as ei:
        c2.verify_list(["x" * 177])                          # the reference overflows data[] and aborts
    assert ei.value.code == dprf.E_DOMAIN
    with pytest.raises(dprf.DprfError) as ei:
        c.verify_list(["z" * (dprf.MAX_PW + 1)])            # no argv string carries it to the reference
    assert ei.value.code == dprf.E_PWLEN
    with pytest.raises(dprf.DprfError):
        c2.search_range(LOWER, 3, 26 ** 3 - 5, 10)


def test_never_matches_and_empty_inputs(dprf):
    f = ["pdf", "2", "4", "128", "-4", "1", "16", "11" * 16, "32", "22" * 32, "32", "33" * 32]
    c = dprf.Context(f)
    assert c.flags & dprf.FLAG_NEVER_MATCHES
    hits, n, st = c.search_range(LOWER, 3, 0, 26 ** 3)
    assert hits == [] and n == 0 and st["candidates"] == 26 ** 3
    c2 = dprf.Context(["pdf", "1", "2", "40", "-64", "1", "16", "11" * 16, "32", "22" * 32, "32", "33" * 32])
    assert c2.verify_list([]) == ([], 0, c2.verify_list([])[2])
    assert c2.search_range(LOWER, 2, 0, 0)[1] == 0


def test_domain_streams_rejected(dprf):
    with pytest.raises(dprf.DprfError) as ei:
        dprf.Context(["odt", "1.2", "11" * 32, "22" * 16, "33" * 16, "44" * 17, "17"])
    assert ei.value.code == dprf.E_DOMAIN
    with pytest.raises(dprf.DprfError) as ei:
        dprf.Context(["pdf", "2", "3", "64", "-4", "1", "16", "11" * 16, "32", "22" * 32, "32", "33" * 32])
    assert ei.value.code == dprf.E_DOMAIN


def test_many_hits_overflow_and_order(dprf, streams, hitsets):
    """The ODT -e 2-byte check has ~2^-16 false positives: a 26^4 scan has 10 (reference, Appendix A)."""
    key = "odt_testdoc_e/lower^4"
    if key not in hitsets:
        pytest.skip("slow golden scan not generated")
    c = ctx_for(dprf, streams, "odt_testdoc_e")
    hits, n, _ = c.search_range(LOWER, 4, 0, 26 ** 4)
    assert hits == hitsets[key]["hits"] and n == 10
    hits3, n3, _ = c.search_range(LOWER, 4, 0, 26 ** 4, cap=3)
    assert n3 == 10 and hits3 == hitsets[key]["hits"][:3]


def test_stop_on_first_returns_lowest(dprf, streams):
    c = ctx_for(dprf, streams, "odt_testdoc_e")
    hits, n, st = c.search_range(LOWER, 4, 0, 26 ** 4, stop_on_first=True, cap=1)
    assert hits == [27692]


def test_range_split_consistency(dprf, streams):
    """A keyspace scanned in one call == the same keyspace scanned in ragged pieces (chunk seams)."""
    c = ctx_for(dprf, streams, "pdf_synth_r4_alnum")
    total = 62 ** 3
    whole, n, _ = c.search_range(ALNUM, 3, 0, total)
    pieces, s = [], 0
    for step in [1, 7, 4095, 100000, total]:
        k = min(step, total - s)
        if k <= 0:
            break
        pieces += c.search_range(ALNUM, 3, s, k)[0]
        s += k
    assert s == total and pieces == whole and len(whole) >= 1


@pytest.mark.parametrize("name", ["pdf_synth_r2_key", "pdf_synth_r3_l40_cab"])
def test_r2_ragged_ranges(dprf, streams, name):
    """R2-R4 workgroups take several batches of 64 candidates each (k_pdf_r24: R2_BATCHES / R34_BATCHES, a key
    wave handing keys to an RC4 wave per batch): counts that are not a multiple of a workgroup's candidates, and
    a start that is not aligned to one, give the same hits and counted candidates."""
    c = ctx_for(dprf, streams, name)
    pw = streams[name]["password"]
    idx = 0
    for ch in pw:
        idx = idx * 26 + LOWER.index(ch)
    total = 26 ** len(pw)
    whole, n, st = c.search_range(LOWER, len(pw), 0, total)
    assert idx in whole and st["candidates"] == total
    pieces, s = [], 0
    for step in [1, 63, 65, 255, 257, 1000, 4097, total]:
        k = min(step, total - s)
        if k <= 0:
            break
        h, _, st = c.search_range(LOWER, len(pw), s, k)
        assert st["candidates"] == k
        pieces += h
        s += k
    assert s == total and pieces == whole
    hits, _, _ = c.search_range(LOWER, len(pw), idx - 5, 11, stop_on_first=True, cap=1)
    assert hits == [idx]


def test_list_mode_equals_range_mode(dprf, streams):
    from dprf_amd import brute_force as bf
    c = ctx_for(dprf, streams, "pdf_synth_r5_alnum")
    start, count = 62 ** 3 - 20000, 20000
    rng_hits, _, _ = c.search_range(ALNUM, 3, start, count)
    words = [bf._index_to_password(start + i, ALNUM, 3) for i in range(count)]
    lst_hits, _, _ = c.verify_list(words)
    assert [start + i for i in lst_hits] == rng_hits


def test_brute_force_module_end_to_end(dprf, streams):
    from dprf_amd import brute_force as bf
    assert bf.init(streams["pdf_synth_r3_l128_abc"]["stream"], 3, None, devices=[0]) == (1, "abc")
    assert bf.init(streams["pdf_testdoc_r2"]["stream"], 2, None, devices=[0]) == (0, "default_password_allocation")
    assert bf.init(streams["office_testdoc"]["stream"], 0, ["x", "password", "y"], devices=[0]) == (1, "password")


def test_multi_device_rounds_on_one_gpu(dprf, streams, monkeypatch):
    """The multi-device code paths (one library context over a device list, one worker thread + stream per
    entry) run here with the device list repeated on the same GPU: same answers as one device, and the
    lowest hit wins when several devices' chunks hold hits."""
    from dprf_amd import brute_force as bf
    from dprf_amd import client as cl
    from dprf_amd import payload as pl
    monkeypatch.setattr(bf, "FIRST_ROUND", 4096)
    monkeypatch.setattr(bf, "ROUND_SECONDS", 0.0)
    monkeypatch.setattr(bf, "ROUND_CHUNKS", 0)
    s = streams["pdf_synth_r3_l128_abc"]["stream"]
    for devs in ([0], [0, 0], [0, 0, 0]):
        assert bf.init(s, 3, None, devices=devs) == (1, "abc")
    e = streams["odt_testdoc_e"]["stream"]          # [a-z]^4 holds 10 hits of the 2-byte check
    want = bf.init(e, 4, None, devices=[0])
    assert bf.init(e, 4, None, devices=[0, 0, 0]) == want == (1, "bozc")
    pws = ["zzzz", "yvgl", "aaaa", "bozc", "password"]
    assert bf.init(e, 0, pws, devices=[0, 0]) == (1, "yvgl")
    # GPU client verifier over a two-device context: the lowest list index that verifies
    ver = cl.GpuVerifier([0, 0])
    blob, offs = pl._pack(pws)
    assert ver(e, blob, offs) == (1, "yvgl")
    ver.close()


def test_multi_device_context_equals_one_device(dprf, streams):
    """dprf_ctx_create_devices({0,0}): two worker threads and streams on the one GPU share each call's chunk
    cursor.  ODF -e over 2^24 alnum^5 indices (4+ launches, ~256 false hits of the 2-byte check): the
    merged hit set equals one device's, and stop_on_first returns the lowest of them on both."""
    from dprf_amd import brute_force as bf
    fields = bf.parse_verification_data(streams["odt_testdoc_e"]["stream"])
    start, count = 62 ** 5 // 3, 1 << 24
    res = {}
    for devs in ([0], [0, 0]):
        with dprf.Context(fields, devices=devs) as c:
            assert c.devices == devs
            hits, n, st = c.search_range(ALNUM, 5, start, count, cap=1 << 12)
            assert st["candidates"] == count and st["devices"] == len(devs) and st["launches"] >= 4
            assert n == len(hits) and n > 16
            fh, _, fst = c.search_range(ALNUM, 5, start, count, stop_on_first=True, cap=1)
            assert fh == hits[:1]
            assert fst["candidates"] >= fh[0] - start + 1     # everything below the lowest hit was verified
            res[tuple(devs)] = hits
    assert res[(0,)] == res[(0, 0)]


def test_small_call_spreads_over_every_device(dprf, streams):
    """a call far smaller than a device's first chunk (a 20,000-candidate client payload; Office's first
    chunk is 2^19) is split over every device of the context -- each lane of a {0,0,0,0} context launches at least
    once (dprf_ctx_last_call_devices) -- with the same hits as one device."""
    from dprf_amd import brute_force as bf
    fields = bf.parse_verification_data(streams["office_testdoc"]["stream"])
    rng = random.Random(9)
    words = ["".join(rng.choice(LOWER) for _ in range(5)) for _ in range(20000)]
    words[17001] = "password"
    for devs in ([0], [0, 0, 0, 0]):
        with dprf.Context(fields, devices=devs) as c:
            hits, nh, st = c.verify_list(words)
            assert hits == [17001] and st["candidates"] == len(words)
            per = c.last_call_devices()
            assert [d["device"] for d in per] == devs
            assert all(d["launches"] >= 1 and d["candidates"] > 0 for d in per), per
            assert sum(d["candidates"] for d in per) == len(words)
            assert all(0 <= d["first_ms"] <= d["finish_ms"] for d in per), per
    # range mode, a multi-launch call: the per-device records add up to the call
    with dprf.Context(bf.parse_verification_data(streams["odt_testdoc_e"]["stream"]), devices=[0, 0]) as c:
        _, _, st = c.search_range(ALNUM, 5, 0, 1 << 23)
        per = c.last_call_devices()
        assert sum(d["candidates"] for d in per) == 1 << 23 and sum(d["launches"] for d in per) == st["launches"]
        assert all(d["launches"] >= 1 for d in per), per


def test_concurrent_calls_on_one_context_are_serialised(dprf, streams):
    """Calls on the same context from several threads (ctypes drops the GIL) are serialised by the library:
    each thread gets exactly the single-threaded hit set and candidate count."""
    import threading
    from dprf_amd import brute_force as bf
    fields = bf.parse_verification_data(streams["odt_testdoc_e"]["stream"])
    start, count = 62 ** 5 // 2, 1 << 22
    with dprf.Context(fields, devices=[0, 0]) as c:
        want, nwant, _ = c.search_range(ALNUM, 5, start, count, cap=1 << 12)
        out = [None] * 4

        def run(k):
            out[k] = c.search_range(ALNUM, 5, start, count, cap=1 << 12)

        th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for hits, n, st in out:
            assert hits == want and n == nwant and st["candidates"] == count


def test_stop_on_first_lowest_across_blocks_and_launches(dprf, streams):
    """The right password planted at several list positions spread over blocks and launches (Office: 2^19
    candidates per launch): stop_on_first answers the lowest position, on one and on two devices, whatever
    order the workgroups run in (a block is skipped only when its lowest index is above the lowest hit)."""
    rng = random.Random(5)
    n = (1 << 19) + 3000
    words = [("".join(rng.choice(LOWER) for _ in range(6))) for _ in range(n)]
    plant = [70001, 262143, 524290, n - 1]
    for k in plant:
        words[k] = "password"
    fields_stream = streams["office_testdoc"]["stream"]
    from dprf_amd import brute_force as bf
    fields = bf.parse_verification_data(fields_stream)
    for devs in ([0], [0, 0]):
        with dprf.Context(fields, devices=devs) as c:
            hits, nh, st = c.verify_list(words)
            assert hits == plant and nh == len(plant) and st["launches"] >= 2
            fh, _, fst = c.verify_list(words, stop_on_first=True, cap=1)
            assert fh == [plant[0]] and fst["candidates"] >= plant[0] + 1


def test_list_status_marks_only_the_invalid_candidates(dprf, streams):
    """The GPU client drops candidates the format cannot take instead of failing the payload."""
    from dprf_amd import client as cl
    from dprf_amd import payload as pl
    s = streams["office_testdoc"]["stream"]
    pws = ["x", "", "bad\x00nul", "password", "y" * 40, "z" * (dprf.MAX_PW + 1)]
    blob, offs = pl._pack(pws)
    with dprf.Context(__import__("dprf_amd.brute_force", fromlist=["x"]).parse_verification_data(s)) as c:
        st = c.list_status(blob, offs)
        assert [int(v) for v in st] == [0, dprf.E_DOMAIN, dprf.E_INVALID, 0, 0, dprf.E_PWLEN]
    ver = cl.GpuVerifier([0])
    assert ver(s, blob, offs) == (1, "password")
    assert ver.skipped == 3
    ver.close()


@pytest.mark.parametrize("name,length,skipped", [("odt_long_e_200", 200, 0), ("pdf_r6_long176", 176, 0),
                                                 ("pdf_r6_long176", 176, 1)])
def test_gpu_client_verifies_long_payloads(dprf, long_verdicts, name, length, skipped):
    """the GPU client drops no candidate the reference verifies -- a payload of 200-byte ODF candidates
    (and 176-byte R6 ones) is verified whole, the document's password among them is found.  Only what the reference
    cannot verify is skipped: a 200-byte R6 candidate aborts the reference (data[] overflow)."""
    from dprf_amd import client as cl
    from dprf_amd import payload as pl
    d = long_verdicts[name]
    rng = random.Random(length)
    pws = ["".join(rng.choice(ALNUM) for _ in range(length)) for _ in range(500)]
    pws[321] = d["password"]
    if skipped:
        pws[17] = "q" * 200
    blob, offs = pl._pack(pws)
    ver = cl.GpuVerifier([0])
    assert ver(d["stream"], blob, offs) == (1, d["password"])
    assert ver.skipped == skipped and ver.verified == len(pws)
    ver.close()


def test_calls_leave_the_callers_device_alone(dprf, streams):
    """every entry point restores the calling thread's HIP device (hipGetDevice through ctypes on
    libamdhip64, which is what torch.cuda.current_device() reads).  With more than one GPU the caller sits on the LAST
    device and the context spans every device, so a call that moved it would be seen."""
    import ctypes
    dprf.lib()                                                       # libdprf.so pulls in the HIP runtime
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        hip = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so")
    cur = ctypes.c_int(-1)

    def get():
        assert hip.hipGetDevice(ctypes.byref(cur)) == 0
        return cur.value
    ndev = dprf.device_count()
    assert hip.hipSetDevice(ndev - 1) == 0
    before = get()
    from dprf_amd import brute_force as bf
    fields = bf.parse_verification_data(streams["pdf_synth_r5_cat"]["stream"])
    c = dprf.Context(fields, devices=list(range(ndev)) if ndev > 1 else [0, 0])
    assert get() == before
    c.search_range(LOWER, 3, 0, 26 ** 3)
    assert get() == before
    c.verify_list(["cat", "x" * 100])
    assert get() == before
    with pytest.raises(dprf.DprfError):
        c.search_range(LOWER, 33, 0, 1)
    assert get() == before
    c.close()
    assert get() == before

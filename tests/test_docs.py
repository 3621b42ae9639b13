"""Self-generated documents (tests/docgen.py, fixtures from tests/golden/make_docs.py): the parsers, the
oracle and the GPU engine against the REFERENCE verifiers on the same files.

Every fixture value was produced by the reference: the verifier streams also by its own office2john.py /
pdf2john.py where they run (docs.json "reference_parser_agrees"), verdicts by its verifier executables,
hit sets by its verify() over the whole [a-z]^3 keyspace."""
import os
import tempfile

import pytest

from conftest import GOLDEN, load_golden

LOWER = "abcdefghijklmnopqrstuvwxyz"
DOCS = os.path.join(GOLDEN, "docs")


@pytest.fixture(scope="module")
def docs():
    return load_golden("docs.json")


def _cases(docs_json=None):
    d = docs_json or load_golden("docs.json")
    return [(name, sk) for name in sorted(d) for sk in sorted(d[name]["streams"])]


def _fields(stream):
    import contextlib
    import io
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def test_parsers_reproduce_fixture_streams(docs):
    from dprf_amd.parsers import odt2hashes, office2john, pdf2john
    for name, e in docs.items():
        path = os.path.join(DOCS, name)
        if e["kind"] == "docx":
            got = {"std": office2john.get_hash(path)}
        elif e["kind"] == "odt":
            got = {"std": odt2hashes.get_hashes(path, False), "e": odt2hashes.get_hashes(path, True)}
        else:
            got = {"std": pdf2john.get_hash(path)}
        assert got == {k: v["stream"] for k, v in e["streams"].items()}, name
        assert e["reference_parser_agrees"] or e["kind"] == "odt"


def test_writers_are_deterministic(docs):
    import docgen
    with tempfile.TemporaryDirectory() as t:
        for name, e in docs.items():
            p = os.path.join(t, name)
            w = {"docx": docgen.write_docx, "odt": docgen.write_odt, "pdf": docgen.write_pdf}[e["kind"]]
            w(p, e["password"], e["seed"], **e["kwargs"])
            assert open(p, "rb").read() == open(os.path.join(DOCS, name), "rb").read(), name


@pytest.mark.parametrize("name,sk", _cases())
def test_oracle_matches_reference_on_documents(oracle, docs, name, sk):
    s = docs[name]["streams"][sk]
    ctx = oracle.Ctx(s["stream"])
    for cand, ref in s["verdicts"]:
        assert int(ctx.verify(cand.encode())) == ref, (name, sk, cand)
    if docs[name]["kind"] != "docx":           # Office: 17,576 x 50k SHA-1 is the GPU test's job
        hits, _ = ctx.search_range(LOWER, 3, 0, 26 ** 3)
        assert hits == s["hitset"]["hits"], (name, sk)


@pytest.mark.gpu
@pytest.mark.parametrize("name,sk", _cases())
def test_gpu_recovers_reference_hitset_on_documents(docs, name, sk):
    """The recovered-password set over [a-z]^3 equals the reference verifier's, bit for bit."""
    from dprf_amd import _lib
    s = docs[name]["streams"][sk]
    with _lib.Context(_fields(s["stream"]), device=0) as ctx:
        hits, n, st = ctx.search_range(LOWER, 3, 0, 26 ** 3)
        assert hits == s["hitset"]["hits"] and n == len(hits), (name, sk)
        assert st["candidates"] == 26 ** 3
        # list mode over the same candidates agrees
        pws = ["".join(t) for t in __import__("itertools").product(LOWER, repeat=3)]
        lh, _, _ = ctx.verify_list(pws)
        assert lh == s["hitset"]["hits"]


@pytest.mark.gpu
def test_brute_force_cli_recovers_document_passwords(docs):
    """The module CLI surface end to end: document -> parser -> GPU range search (brute_force.py:266-298)."""
    import contextlib
    import io
    from dprf_amd import brute_force
    for name, e in docs.items():
        doc_type = {"docx": "1", "odt": "2", "pdf": "3"}[e["kind"]]
        with contextlib.redirect_stdout(io.StringIO()):
            found, pw = brute_force.main([doc_type, os.path.join(DOCS, name), "-pr", "3"])
        assert (found, pw) == (1, e["password"]), name


RANDOM_DOCS = [("docx", {}), ("odt", {}), ("pdf", {"R": 2, "length": 40}), ("pdf", {"R": 3, "length": 128}),
               ("pdf", {"R": 3, "length": 40}), ("pdf", {"R": 4, "length": 128, "meta": False}),
               ("pdf", {"R": 5, "length": 256}), ("pdf", {"R": 6, "length": 256})]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,kw", RANDOM_DOCS, ids=lambda v: v if isinstance(v, str) else
                         "-".join("%s%s" % kv for kv in sorted(v.items())))
def test_gpu_random_documents_vs_oracle(oracle, kind, kw):
    """Documents with fresh random salts / IDs / IVs and a random [a-z]^3 password (seeded, written by
    tests/docgen.py and parsed by dprf_amd/parsers): the GPU hit set over the whole [a-z]^3 keyspace holds
    the password and the oracle confirms every hit; the oracle's own scan of the keyspace equals it where
    that takes well under a second (PDF R2-R5), elsewhere 300 random non-hits are confirmed as misses."""
    import random
    import zlib
    import docgen
    from dprf_amd import _lib
    from dprf_amd.parsers import odt2hashes, office2john, pdf2john
    rng = random.Random(zlib.crc32(repr((kind, sorted(kw.items()))).encode()))
    full_scan = kind == "pdf" and kw["R"] <= 5
    with tempfile.TemporaryDirectory() as t:
        for trial in range(2):
            pw = "".join(rng.choice(LOWER) for _ in range(3))
            seed = rng.randrange(1 << 30)
            path = os.path.join(t, "doc%d.%s" % (trial, kind))
            if kind == "docx":
                docgen.write_docx(path, pw, seed)
                streams = [office2john.get_hash(path)]
            elif kind == "odt":
                docgen.write_odt(path, pw, seed)
                streams = [odt2hashes.get_hashes(path, False), odt2hashes.get_hashes(path, True)]
            else:
                docgen.write_pdf(path, pw, seed, **kw)
                streams = [pdf2john.get_hash(path)]
            idx = 0
            for ch in pw:
                idx = idx * 26 + LOWER.index(ch)
            for stream in streams:
                octx = oracle.Ctx(stream)
                with _lib.Context(_fields(stream), device=0) as ctx:
                    hits, n, st = ctx.search_range(LOWER, 3, 0, 26 ** 3)
                assert st["candidates"] == 26 ** 3 and n == len(hits)
                assert idx in hits, (kind, kw, pw, seed)
                word = lambda h: (LOWER[h // 676] + LOWER[h // 26 % 26] + LOWER[h % 26]).encode()
                for h in hits:
                    assert octx.verify(word(h)) == 1, (kind, kw, h)
                if full_scan:
                    want, _ = octx.search_range(LOWER, 3, 0, 26 ** 3)
                    assert hits == want, (kind, kw, pw, seed)
                else:
                    hs = set(hits)
                    for h in rng.sample(range(26 ** 3), 300):
                        if h not in hs:
                            assert octx.verify(word(h)) == 0, (kind, kw, h)

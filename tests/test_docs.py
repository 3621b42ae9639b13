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

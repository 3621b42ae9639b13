"""INTEGRATION.md section 2's ctypes stub -- what a maintainer pastes into the reference's brute_force.py -- run as
written: the python block is extracted from the document, pointed at the in-tree libdprf.so and executed.  CPU: it
loads and declares a prototype for every entry point it calls, matching include/dprf.h's parameter count.  GPU: its
gpu_list / gpu_range / gpu_range_symbols find the planted passwords of generated documents with the reference's
return values."""
import os
import re
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub():
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    sec = doc[doc.index("## 2. Bind the C ABI"):doc.index("## 3.")]
    code = re.search(r"```python\n(.*?)```", sec, re.S).group(1)
    assert 'ctypes.CDLL("libdprf.so")' in code
    code = code.replace('ctypes.CDLL("libdprf.so")', "ctypes.CDLL(%r)" % os.path.join(REPO, "dprf_amd", "libdprf.so"))
    ns = {}
    exec(compile(code, "INTEGRATION.md", "exec"), ns)
    return ns


def test_stub_declares_every_prototype_it_calls():
    ns = _stub()
    hdr = open(os.path.join(REPO, "include", "dprf.h")).read()
    L = ns["_dprf"]
    for name in ("dprf_ctx_create", "dprf_ctx_destroy", "dprf_verify_list", "dprf_search_range", "dprf_search_symbols"):
        decl = re.search(r"\b%s\(([^)]*)\);" % name, hdr, re.S).group(1)
        assert len(getattr(L, name).argtypes) == len(decl.split(",")), name
    for fn in ("gpu_list", "gpu_range", "gpu_range_symbols"):
        assert callable(ns[fn])


def _fields(kind, pw):
    import contextlib
    import io
    import docgen
    from dprf_amd.brute_force import parse_verification_data
    from dprf_amd.parsers import odt2hashes, pdf2john
    with tempfile.TemporaryDirectory() as t:
        if kind == "odt":
            docgen.write_odt(os.path.join(t, "d.odt"), pw, 0x1A7)
            stream = odt2hashes.get_hashes(os.path.join(t, "d.odt"), False)
        else:
            docgen.write_pdf(os.path.join(t, "d.pdf"), pw, 0x1A7, R=4, length=128)
            stream = pdf2john.get_hash(os.path.join(t, "d.pdf"))
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


@pytest.mark.gpu
def test_stub_finds_passwords():
    ns = _stub()
    f = _fields("pdf", "dcba")
    assert ns["gpu_list"](f, ["x", "dcba", "y"]) == (1, "dcba")
    assert ns["gpu_list"](f, ["x", "y"]) == (0, "default_password_allocation")
    assert ns["gpu_range"](f, 4, "abcd") == (1, "dcba")
    assert ns["gpu_range"](f, 3, "abcd") == (0, "default_password_allocation")
    g = _fields("odt", "éa€")
    assert ns["gpu_range_symbols"](g, 3, "aé€") == (1, "éa€")

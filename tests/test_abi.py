"""The C-ABI library loads and exports every symbol include/dprf.h declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest

from conftest import REPO


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "dprf.h")).read()
    return sorted(set(re.findall(r"\b(dprf_[a-z_]+)\s*\(", hdr)))


def test_header_and_python_binding_agree():
    from dprf_amd import _lib
    assert declared_symbols() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    from dprf_amd import _lib
    L = _lib.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    assert L.dprf_abi_version() == _lib.ABI_VERSION


def test_constants_match_header():
    from dprf_amd import _lib
    hdr = open(os.path.join(REPO, "include", "dprf.h")).read()
    consts = dict((k, int(v)) for k, v in re.findall(r"#define (DPRF_\w+) \(?(-?\d+)\)?", hdr))
    assert consts["DPRF_ABI_VERSION"] == _lib.ABI_VERSION
    assert consts["DPRF_E_DOMAIN"] == _lib.E_DOMAIN and consts["DPRF_E_NODEVICE"] == _lib.E_NODEVICE
    assert consts["DPRF_MAX_PW"] == _lib.MAX_PW and consts["DPRF_MAX_PW_RANGE"] == _lib.MAX_PW_RANGE
    assert consts["DPRF_FLAG_NEVER_MATCHES"] == _lib.FLAG_NEVER_MATCHES


def test_no_device_is_an_error_not_a_fallback():
    """Without a GPU, creating a context must fail loudly (DPRF_E_NODEVICE) -- there is no CPU path."""
    from dprf_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.DprfError) as ei:
        _lib.Context(["pdf", "1", "2", "40", "-64", "1", "16", "11" * 16, "32", "22" * 32, "32", "33" * 32])
    assert ei.value.code == _lib.E_NODEVICE


def test_product_does_not_import_the_oracle():
    """Nothing under dprf_amd/ may import, load or execute oracle/ (it is the checker)."""
    for root, _, files in os.walk(os.path.join(REPO, "dprf_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(root, f), errors="replace").read()
                assert "pyoracle" not in src and "liboracle" not in src and "oracle.h" not in src, f


def test_makefile_tracks_every_local_header():
    """Every header a kernel or host source includes is a make dependency and part of the build fingerprint
    (HDRS): round 3 once shipped a stale object because the generated rc4_ksa_asm.h was missing there, so the
    library -- and its dprf_build_id() -- did not change when the header did."""
    import re
    csrc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dprf_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    hdrs = set(re.search(r"^HDRS\s*:=\s*(.*)$", mk, re.M).group(1).split())
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            for inc in re.findall(r'^#include "([^"]+)"', open(os.path.join(csrc, f)).read(), re.M):
                if inc == "build_id.h":
                    continue                      # generated into OBJDIR by the Makefile itself
                assert inc in hdrs, (f, inc)


def test_ctypes_structs_match_the_header_layout(tmp_path):
    """dprf_stats / dprf_device_stats as a C compiler lays them out (include/dprf.h) == the ctypes mirrors (ABI 6
    appended hit_ms and evaluated): sizes and every field offset."""
    import subprocess
    from dprf_amd import _lib
    src = tmp_path / "layout.c"
    fields = {"dprf_stats": [f for f, _ in _lib.Stats._fields_],
              "dprf_device_stats": [f for f, _ in _lib.DeviceStats._fields_]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "dprf.h"', "int main(void) {"]
    for t, fs in fields.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (t, t))
        for f in fs:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (t, f, t, f))
    lines.append("return 0; }")
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n") if ln)
    for t, cls in (("dprf_stats", _lib.Stats), ("dprf_device_stats", _lib.DeviceStats)):
        assert int(got[t]) == ctypes.sizeof(cls), t
        for f, _ in cls._fields_:
            assert int(got["%s.%s" % (t, f)]) == getattr(cls, f).offset, (t, f)

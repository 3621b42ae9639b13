"""A hit stops the other devices' launches while they run (round 6, VERDICT r5 Missing #1 / Next #3).

The reference stops every worker at its next candidate once one has found the password (brute_force.py:111-114,
:140-147).  Before round 6 a device of a multi-device call learned of another device's hit only when one of its own
launches retired, so its launches in flight ran to their end -- up to a whole 12-second R6 launch.  Now a multi-device
stop_on_first call gives every launch two host-mapped words (dprf_hits.h): the lane's hit mirror, and the call's
lowest hit, which a host thread keeps at the minimum of the mirrors (dprf_host.cpp call_watch).

The GPU tests plant the password early in lane 0's first chunk of a call over two and four lanes on the one GPU
({0,0}, {0,0,0,0}: the same protocol as separate GPUs, each lane with its own results buffer and words) and check
that the other lanes -- whose chunks lie entirely above the hit -- verify at most about one generation of resident
workgroups past it (dprf_ctx_last_call_devices `evaluated`, ABI 6), and that the call still returns the lowest hit.
The time from the host first knowing the hit to the call returning (stats wall_ms - hit_ms) is printed and kept in
gpurun_out/stop_push.json for profiles/."""
import contextlib
import io
import json
import os
import tempfile

import pytest

LOWER = "abcdefghijklmnopqrstuvwxyz"
PW = "aaabc"                                   # index 28 of lowercase^5 (11.9 M candidates)
IDX = LOWER.index("b") * 26 + LOWER.index("c")
GEN = 1 << 19                                  # > one generation of resident candidates (ODF 393 k, R6 278 k slots)


def _stream(kind):
    import docgen
    from dprf_amd.parsers import odt2hashes, pdf2john
    with tempfile.TemporaryDirectory() as t:
        if kind == "odt":
            docgen.write_odt(os.path.join(t, "d.odt"), PW, 0x5709)
            return odt2hashes.get_hashes(os.path.join(t, "d.odt"), False)
        docgen.write_pdf(os.path.join(t, "d.pdf"), PW, 0x5709, R=6, length=256)
        return pdf2john.get_hash(os.path.join(t, "d.pdf"))


def _fields(stream):
    from dprf_amd.brute_force import parse_verification_data
    with contextlib.redirect_stdout(io.StringIO()):
        return parse_verification_data(stream)


def test_planted_streams_verify_on_the_oracle(oracle):
    for kind in ("odt", "pdf_r6"):
        octx = oracle.Ctx(_stream(kind))
        assert octx.verify(PW.encode()) == 1 and octx.verify(b"aaabd") == 0, kind


def _record(key, value):
    os.makedirs("gpurun_out", exist_ok=True)
    path = os.path.join("gpurun_out", "stop_push.json")
    d = json.load(open(path)) if os.path.exists(path) else {}
    d[key] = value
    json.dump(d, open(path, "w"), indent=1, sort_keys=True)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["odt", "pdf_r6"])
@pytest.mark.parametrize("lanes", [2, 4])
def test_a_hit_stops_the_other_lanes_launches(kind, lanes):
    from dprf_amd import _lib
    stream = _stream(kind)
    total = 26 ** 5
    with _lib.Context(_fields(stream), devices=[0] * lanes) as ctx:
        hits, nh, st = ctx.search_range(LOWER, 5, 0, total, stop_on_first=True, cap=4)
        per = ctx.last_call_devices()
    assert hits[:1] == [IDX], (kind, lanes, hits)
    assert st["hit_ms"] >= 0 and st["stopped_early"] == 1, st
    others = per[1:]
    assert all(d["launches"] >= 1 for d in others), per          # every lane had a launch in flight above the hit
    for d in others:
        assert d["evaluated"] <= GEN, (kind, lanes, per)
    assert sum(d["evaluated"] for d in per) <= lanes * GEN, per
    after = st["wall_ms"] - st["hit_ms"]
    print("%s %d lanes: hit known at %.1f ms, call returned %.1f ms later; lanes evaluated %s of launched %s"
          % (kind, lanes, st["hit_ms"], after, [d["evaluated"] for d in per], [d["candidates"] for d in per]))
    _record("%s_lanes%d" % (kind, lanes), {"hit_ms": st["hit_ms"], "wall_ms": st["wall_ms"], "after_hit_ms": after,
                                          "evaluated": [d["evaluated"] for d in per],
                                          "launched": [d["candidates"] for d in per]})


@pytest.mark.gpu
def test_a_hit_stops_the_other_lanes_in_list_mode():
    """The same in list mode (a client payload): 2 Mi candidates, the password at list index 5."""
    import numpy as np
    from dprf_amd import _lib
    from dprf_amd.payload import spell_utf8
    stream = _stream("odt")
    n = 1 << 21
    blob, offs = spell_utf8("bcdefghijklmnopqrstuvwxyz", 5, 0, n)   # no 'a': none of them is the password
    words = [blob[int(offs[k]):int(offs[k + 1])] for k in range(8)]
    words[5] = PW.encode()
    head = b"".join(words)
    blob = head + blob[int(offs[8]):]
    offs = offs.copy()
    offs[1:9] = np.cumsum([len(w) for w in words])
    with _lib.Context(_fields(stream), devices=[0, 0]) as ctx:
        hits, _, st = ctx.verify_blob(blob, offs, stop_on_first=True, cap=4)
        per = ctx.last_call_devices()
    assert hits[:1] == [5], hits
    assert per[1]["evaluated"] <= GEN, per
    _record("odt_list_lanes2", {"hit_ms": st["hit_ms"], "wall_ms": st["wall_ms"],
                                "after_hit_ms": st["wall_ms"] - st["hit_ms"],
                                "evaluated": [d["evaluated"] for d in per], "launched": [d["candidates"] for d in per]})


@pytest.mark.gpu
def test_one_lane_reports_the_hit_time():
    from dprf_amd import _lib
    stream = _stream("odt")
    with _lib.Context(_fields(stream), device=0) as ctx:
        hits, _, st = ctx.search_range(LOWER, 5, 0, 1 << 20, stop_on_first=True, cap=4)
        assert hits[:1] == [IDX] and 0 <= st["hit_ms"] <= st["wall_ms"], st
        hits, _, st = ctx.search_range(LOWER, 5, 1 << 20, 1 << 16, stop_on_first=True, cap=4)
        assert hits == [] and st["hit_ms"] == -1, st


@pytest.mark.gpu
def test_a_hit_stops_the_other_lanes_in_a_symbol_window():
    """The same for a device-spelled symbol window (ABI 7): ODF, 2-byte characters, the password early in lane 0's
    first chunk of a 2^22-candidate window on two lanes."""
    import docgen
    from dprf_amd import _lib
    from dprf_amd.parsers import odt2hashes
    cs = "αβγδεζηθικλμνξοπρστυφχψω"
    pw = "ααβγ" + "δε"
    with tempfile.TemporaryDirectory() as t:
        docgen.write_odt(os.path.join(t, "d.odt"), pw, 0x5709)
        stream = odt2hashes.get_hashes(os.path.join(t, "d.odt"), False)
    idx = sum(cs.index(ch) * len(cs) ** (5 - k) for k, ch in enumerate(pw))
    with _lib.Context(_fields(stream), devices=[0, 0]) as ctx:
        hits, _, st = ctx.search_symbols(cs, 6, 0, 1 << 22, stop_on_first=True, cap=4)
        per = ctx.last_call_devices()
    assert hits[:1] == [idx] and st["stopped_early"] == 1, (hits, st)
    assert per[1]["evaluated"] <= GEN, per
    _record("odt_symbols_lanes2", {"hit_ms": st["hit_ms"], "wall_ms": st["wall_ms"],
                                   "after_hit_ms": st["wall_ms"] - st["hit_ms"],
                                   "evaluated": [d["evaluated"] for d in per], "launched": [d["candidates"] for d in per]})

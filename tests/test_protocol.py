"""Work-distribution protocol counterparts (dprf_amd.server / dprf_amd.client / dprf_amd.payload) against
the reference's server.py / client.py behaviour: candidate order (server.py:189-199), payload JSON
(:285-292), client loop and found report (client.py:36-69), heartbeat (:209-238), re-queue of an inactive
client's payload (:241-256).  CPU tests drive the real server and client loop over localhost with a
verifier stub backed by the oracle (the checker); the GPU test runs the real GPU client."""
import itertools
import json
import random
import socket
import threading
import time

import numpy as np
import pytest

from dprf_amd import client as cl
from dprf_amd import payload as pl
from dprf_amd import server as sv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reference_order(cs, n):
    out = []
    for x in range(1, n + 1):
        out.extend("".join(t) for t in itertools.product(cs, repeat=x))
    return out


@pytest.mark.parametrize("cs,n", [("abc", 4), (pl.LOWERCASE, 2), ("xy", 6)])
def test_keyspace_is_server_order(cs, n):
    ref = _reference_order(cs, n)
    ks = pl.Keyspace(cs, n)
    assert ks.total == len(ref)
    got = []
    rng = random.Random(3)
    g = 0
    while g < ks.total:
        step = rng.randint(1, 40)
        for L, s, c in ks.segments(g, step):
            got.extend(ks.password(L, s + k) for k in range(c))
        g += step
    assert got == ref
    for i in rng.sample(range(len(ref)), 20):
        assert ks.global_index(ref[i]) == i


def test_keyspace_facts():
    ks = pl.Keyspace(pl.LOWERCASE, 8)
    assert ks.total == 217180147158
    assert ks.global_index("password") == 129052722139
    assert pl.Keyspace("ab", 3, limit=5).total == 5


@pytest.mark.parametrize("cs,n,g0,cnt", [("abc", 3, 0, 39), (pl.LOWERCASE, 3, 700, 100), ("01", 5, 3, 50)])
def test_build_message_is_json_of_the_payload(cs, n, g0, cnt):
    ks = pl.Keyspace(cs, n)
    segs = ks.segments(g0, cnt)
    raw = pl.build_message("x.pdf:$pdf$*1*2", cs, segs)
    d = json.loads(raw)
    assert d["data"] == "x.pdf:$pdf$*1*2"
    assert d["passwords"] == _reference_order(cs, n)[g0:g0 + cnt]


def _roundtrip(msg_obj, raw=None):
    raw = raw if raw is not None else json.dumps(msg_obj).encode()
    stream, blob, offs = pl.parse_message(raw)
    assert stream == msg_obj["data"]
    assert [pl.candidate(blob, offs, k) for k in range(len(offs) - 1)] == msg_obj["passwords"]
    assert offs.dtype == np.uint64 and len(offs) == len(msg_obj["passwords"]) + 1


def test_parse_message_fast_and_fallback_paths():
    rng = random.Random(11)
    alpha = "abcXYZ019 :,[]{}-_"
    pw = ["".join(rng.choice(alpha) for _ in range(rng.randint(0, 12))) for _ in range(500)]
    _roundtrip({"data": "doc.docx:$office$*2007*20", "passwords": pw})
    # the reference (py2 dict order) may put "passwords" first
    obj = {"passwords": pw[:50], "data": "doc.pdf:$pdf$*4*4"}
    _roundtrip({"data": obj["data"], "passwords": obj["passwords"]}, json.dumps(obj).encode())
    # escapes -> json.loads path (quotes, backslashes, non-ASCII as \\u escapes)
    _roundtrip({"data": 'we"ird\\name.pdf:$pdf$', "passwords": ['a"b', "c\\d", "päss", "€"]})
    _roundtrip({"data": "d:$odt$", "passwords": []})
    _roundtrip({"data": "d:$odt$", "passwords": ["", "", "a"]})


class _OracleVerifier:
    """verify(stream, blob, offsets) -> (found, password) on the CPU oracle (test infrastructure)."""

    def __init__(self, oracle):
        self.oracle = oracle
        self.ctx = None
        self.seen = []

    def __call__(self, stream, blob, offsets):
        if self.ctx is None:
            self.ctx = self.oracle.Ctx(stream)
        pws = [pl.candidate(blob, offsets, k) for k in range(len(offsets) - 1)]
        self.seen.extend(pws)
        for p in pws:
            if self.ctx.verify(p.encode()):
                return 1, p
        return 0, None


def _run_server(srv):
    out = {}
    th = threading.Thread(target=lambda: out.setdefault("pw", srv.run("127.0.0.1", 0)), daemon=True)
    th.start()
    assert srv.bound.wait(10)
    return th, out


def test_server_client_end_to_end_finds_password(streams, oracle):
    d = streams["pdf_synth_r5_cat"]
    srv = sv.Server(d["stream"], password_range=3, payload_size=997, heartbeat_port=_free_port(), quiet=True)
    th, out = _run_server(srv)
    ver = _OracleVerifier(oracle)
    rc, pw = cl.connect_to_server("127.0.0.1", srv.address[1], "client-1", ver, quiet=True)
    th.join(10)
    assert (rc, pw) == (0, "cat")
    assert out["pw"] == "cat" and srv.found
    # the client saw exactly the server's order up to the payload that held the password
    ref = _reference_order(pl.LOWERCASE, 3)
    assert ver.seen == ref[:len(ver.seen)] and "cat" in ver.seen


def test_server_exhausts_keyspace_and_two_clients_split_it(streams, oracle):
    d = streams["pdf_synth_r5_cat"]
    srv = sv.Server(d["stream"], password_range=2, payload_size=50, heartbeat_port=_free_port(), quiet=True)
    th, out = _run_server(srv)
    vers = [_OracleVerifier(oracle), _OracleVerifier(oracle)]
    res = [None, None]
    ths = [threading.Thread(target=lambda k=k: res.__setitem__(
        k, cl.connect_to_server("127.0.0.1", srv.address[1], "c%d" % k, vers[k], quiet=True))) for k in range(2)]
    [t.start() for t in ths]
    [t.join(30) for t in ths]
    th.join(10)
    assert out["pw"] is None and not srv.found
    assert [r[0] for r in res] == [1, 1]          # "No data received from server. Exiting." (client.py:48-50)
    seen = sorted(vers[0].seen + vers[1].seen, key=lambda p: (len(p), p))
    assert seen == _reference_order(pl.LOWERCASE, 2)
    assert srv.counter == 26 + 26 * 26


def test_heartbeat_and_inactive_requeue(streams):
    d = streams["pdf_synth_r5_cat"]
    hb = _free_port()
    srv = sv.Server(d["stream"], password_range=2, payload_size=10, heartbeat_port=hb, quiet=True,
                    inactive_after=0.5, cleanup_every=0.3)
    th, out = _run_server(srv)
    # a client takes one payload and disappears
    c = socket.create_connection(srv.address)
    c.sendall(cl.prepare_message("ghost", False, None))
    c.shutdown(socket.SHUT_WR)
    first = json.loads(cl.recvall(c))
    c.close()
    assert first["passwords"] == _reference_order(pl.LOWERCASE, 2)[:10]
    # heartbeat answers {"found": false}
    time.sleep(0.2)
    h = socket.create_connection(("127.0.0.1", hb))
    h.sendall(cl.prepare_message("ghost", None, None, True))
    h.shutdown(socket.SHUT_WR)
    assert json.loads(cl.recvall(h)) == {"found": False}
    h.close()
    time.sleep(1.5)                                   # ghost is dropped, its payload re-queued
    assert all(x.id != "ghost" for x in srv.clients)
    seen = []

    def ver(stream, blob, offs):
        seen.extend(pl.candidate(blob, offs, k) for k in range(len(offs) - 1))
        return 0, None
    rc, _ = cl.connect_to_server("127.0.0.1", srv.address[1], "late", ver, quiet=True)
    th.join(10)
    assert rc == 1
    assert sorted(seen) == sorted(_reference_order(pl.LOWERCASE, 2))


@pytest.mark.gpu
def test_gpu_client_against_server(streams):
    """The GPU client (libdprf list mode) finds the password the server's payloads hold."""
    for name, pr, ps in (("pdf_synth_r4_meta0_dog", 3, 4096), ("office_synth_ok", 2, 300), ("odt_synth_std_zq", 2, 256)):
        d = streams[name]
        srv = sv.Server(d["stream"], password_range=pr, payload_size=ps, heartbeat_port=_free_port(), quiet=True)
        th, out = _run_server(srv)
        ver = cl.GpuVerifier([0])
        rc, pw = cl.connect_to_server("127.0.0.1", srv.address[1], "gpu", ver, quiet=True)
        ver.close()
        th.join(10)
        assert (rc, pw) == (0, d["password"]), name
        assert out["pw"] == d["password"]


class _FakeCtx:
    """Stand-in for _lib.Context on CPU (test infrastructure): the oracle's verdicts, and the library's
    list-mode rule that one invalid candidate fails the whole call (dprf_verify_list) while
    dprf_list_status marks it."""

    def __init__(self, fields, devices=None):
        import pyoracle
        self.c = pyoracle.Ctx(fields)
        self.fields = fields
        self.devices = devices

    def _status(self, p):
        """dprf_list_status's rules (include/dprf.h, ABI 5): NUL; longer than an argv string; Office "" or invalid
        UTF-8; PDF R6 over 176 bytes"""
        from dprf_amd import _lib
        if b"\x00" in p:
            return _lib.E_INVALID
        if len(p) > _lib.MAX_PW:
            return _lib.E_PWLEN
        if self.fields[0] == "office":
            try:
                p.decode("utf-8")
            except UnicodeDecodeError:
                return _lib.E_DOMAIN
            return _lib.E_DOMAIN if not p else 0
        if self.fields[0] == "pdf" and self.fields[2] == "6" and len(p) > _lib.MAX_PW_R6:
            return _lib.E_DOMAIN
        return 0

    def list_status(self, blob, offsets):
        b = bytes(blob)
        return np.array([self._status(b[int(offsets[k]):int(offsets[k + 1])]) for k in range(len(offsets) - 1)],
                        dtype=np.int8)

    def verify_blob(self, blob, offsets, stop_on_first=False, cap=1 << 16):
        from dprf_amd import _lib
        st = self.list_status(blob, offsets)
        if (st != 0).any():
            k = int(np.flatnonzero(st)[0])
            raise _lib.DprfError(int(st[k]), "candidate %d invalid" % k)
        b = bytes(blob)
        hits = [k for k in range(len(offsets) - 1) if self.c.verify(b[int(offsets[k]):int(offsets[k + 1])])]
        return hits[:cap], len(hits), {}

    def close(self):
        pass


def test_gpu_verifier_drops_invalid_candidates_instead_of_failing(streams, monkeypatch):
    """a payload with a candidate the format cannot take (NUL, empty Office password, > 32 UTF-16
    units) is verified without it -- the reference fails such a candidate in its own process -- rather than
    crashing every client it is re-queued to.  The lowest VALID index that verifies is the answer."""
    from dprf_amd import _lib
    monkeypatch.setattr(_lib, "Context", _FakeCtx)
    s = streams["office_testdoc"]["stream"]
    ver = cl.GpuVerifier(devices=[0])
    pws = ["x", "", "bad\x00nul", "y" * 40, "z" * (_lib.MAX_PW + 1), "password", "password"]
    blob, offs = pl._pack(pws)
    assert ver(s, blob, offs) == (1, "password")
    assert ver.skipped == 3 and ver.verified == len(pws)          # a 40-character candidate is verified (round 4)
    blob, offs = pl._pack(["a", "b"])
    assert ver(s, blob, offs) == (0, None)          # the valid-only path leaves clean payloads alone
    ver.close()


def test_server_survives_a_client_that_dies_before_reading(streams):
    """sendall to a client that is gone must not end the server; the payload stays for the next
    connection."""
    srv = sv.Server(streams["office_testdoc"]["stream"], password_range=2, payload_size=50, quiet=True,
                    heartbeat_port=0)
    msg, segs = srv.prepare_data_for_transfer()

    class Once:
        """A client socket that sends its request, then is gone before the answer."""

        def recv(self, n):
            if getattr(self, "done", False):
                return b""
            self.done = True
            return json.dumps({"found": False, "correct_password": "", "id": "c1"}).encode()

        def settimeout(self, t):
            pass

        def shutdown(self, how):
            pass

        def sendall(self, m):
            raise BrokenPipeError("client went away")

        def close(self):
            pass

    found, sent = srv.handle_connection(Once(), ("127.0.0.1", 1), msg, segs)
    assert (found, sent) == (False, False)
    assert srv.clients == [] and "c1" not in srv.processed_passwords
    srv.pool.shutdown(wait=False)


def _gpu_clients(port, hb, n, cwd):
    """n real GPU client processes (python -m dprf_amd.client, one library context each on device 0), as
    configs[4] runs them; returns their summary JSON lines."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, "-m", "dprf_amd.client", "127.0.0.1", str(port), "--devices", "0",
                               "--heartbeat-port", str(hb), "--quiet"], cwd=cwd, env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for _ in range(n)]
    out = []
    for p in procs:
        txt, _ = p.communicate(timeout=100)
        lines = [ln for ln in txt.splitlines() if ln.startswith("{")]
        assert lines, txt
        out.append(json.loads(lines[-1]))
    return out


@pytest.mark.gpu
def test_config5_two_gpu_clients_office_real_shape(tmp_path):
    """configs[4] at its shape: an Office 2007 document written by tests/docgen.py whose
    4-letter password sits in the last quarter of the server's lengths-1..4 order, served with -ps 65536 to TWO
    GPU client processes on device 0.  The server's answer is the planted password; its global index in server
    order is the planted one; both clients verified payloads; the oracle (the checker) accepts the password.
    Uniqueness -- that no lower index also verifies -- is not re-derived on the CPU (475k Office verifies): the
    check compares a 20-byte SHA-1 digest, so a second hit in the lower indices is a ~2^-141 event."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    import docgen
    import pyoracle
    from dprf_amd.parsers import office2john
    pw = "uqyz"
    ks = pl.Keyspace(pl.LOWERCASE, 4)
    g = ks.global_index(pw)
    assert g >= 3 * ks.total // 4
    doc = str(tmp_path / "config5.docx")
    docgen.write_docx(doc, pw, seed=5)
    stream = office2john.get_hash(doc).strip()
    assert pyoracle.Ctx(stream).verify(pw.encode())
    srv = sv.Server(stream, password_range=4, payload_size=65536, heartbeat_port=_free_port(), quiet=True)
    sent = []
    orig = srv.handle_connection

    def handle(client, address, message, segs):
        r = orig(client, address, message, segs)
        if r[1]:
            sent.append(segs)
        return r
    srv.handle_connection = handle
    th, out = _run_server(srv)
    res = _gpu_clients(srv.address[1], srv.heartbeat_port, 2, os.path.dirname(os.path.dirname(__file__)))
    th.join(30)
    assert out["pw"] == pw and srv.found
    assert ks.global_index(out["pw"]) == g
    assert all(r["verified"] > 0 for r in res), res
    assert sorted(r["password"] is not None for r in res) == [False, True], res
    # payloads went out in server order and the one that holds g was among them
    starts = [ks.global_index(ks.password(s[0][0], s[0][1])) for s in sent]
    assert starts == sorted(starts)
    assert any(st <= g < st + sum(c for _, _, c in s) for st, s in zip(starts, sent))


@pytest.mark.gpu
def test_config5_office_testdoc_first_mi_of_pr8_no_hit(streams):
    """The reference's Office test document over the first 2^20 indices of the server's -pr 8 order (password
    'password' lies at 129,052,722,139): no hit, and every payload verified exactly once by the two GPU
    clients -- the server acknowledges 2^20 candidates, the clients' counts sum to 2^20, the payloads tile
    [0, 2^20) without overlap."""
    import os
    s = streams["office_testdoc"]["stream"]
    n = 1 << 20
    srv = sv.Server(s, password_range=8, payload_size=65536, heartbeat_port=_free_port(), quiet=True,
                    max_candidates=n)
    sent = []
    orig = srv.handle_connection

    def handle(client, address, message, segs):
        r = orig(client, address, message, segs)
        if r[1]:
            sent.append(segs)
        return r
    srv.handle_connection = handle
    th, out = _run_server(srv)
    res = _gpu_clients(srv.address[1], srv.heartbeat_port, 2, os.path.dirname(os.path.dirname(__file__)))
    th.join(30)
    assert out["pw"] is None and not srv.found
    assert sum(r["verified"] for r in res) == n and all(r["verified"] > 0 for r in res), res
    assert srv.counter == n
    ks = pl.Keyspace(pl.LOWERCASE, 8)
    spans = sorted((ks.global_index(ks.password(sg[0][0], sg[0][1])), sum(c for _, _, c in sg)) for sg in sent)
    pos = 0
    for st, c in spans:
        assert st == pos
        pos += c
    assert pos == n


@pytest.mark.gpu
def test_gpu_client_finds_passwords_at_payload_and_length_edges(tmp_path):
    """Planted passwords at the edges of the server's order (server.py:189-199): the last and first candidate of a
    payload, the last candidate of one length and the first of the next, and the keyspace's very last candidate --
    each in a fresh PDF R4 document (tests/docgen.py), found by the real GPU client through the server."""
    import docgen
    from dprf_amd.parsers import pdf2john
    ks = pl.Keyspace(pl.LOWERCASE, 3)
    ps = 1000
    for g in (5 * ps - 1, 5 * ps, ks.sizes[0] + ks.sizes[1] - 1, ks.sizes[0] + ks.sizes[1], ks.total - 1):
        L = next(L for L, s, c in ks.segments(g, 1))
        start = sum(ks.sizes[:L - 1])
        pw = ks.password(L, g - start)
        assert ks.global_index(pw) == g
        path = str(tmp_path / ("edge%d.pdf" % g))
        docgen.write_pdf(path, pw, g, R=4, length=128)
        srv = sv.Server(pdf2john.get_hash(path), password_range=3, payload_size=ps, heartbeat_port=_free_port(),
                        quiet=True)
        th, out = _run_server(srv)
        ver = cl.GpuVerifier([0])
        rc, found = cl.connect_to_server("127.0.0.1", srv.address[1], "gpu", ver, quiet=True)
        ver.close()
        th.join(10)
        assert (rc, found) == (0, pw) and out["pw"] == pw, (g, pw, rc, found)

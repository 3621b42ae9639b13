#!/usr/bin/env python3
"""Distributed Document Password Brute-Force Framework Client, GPU-backed -- Python-3 counterpart of
/root/reference/src/client.py with the same CLI and protocol:

* ``python -m dprf_amd.client tcp_ip tcp_port`` (client.py:118-162); a uuid4 identifies the instance.
* loop (connect_to_server, client.py:36-69): connect, send ``{"found", "correct_password", "id"}``,
  half-close, read the whole answer; no answer -> exit(1); otherwise verify the payload's passwords
  against its verifier stream; repeat until found, then report the password once more.
* heartbeat thread: ``{"id"}`` to port 31337 every 20 s (client.py:101-116).

The payload goes straight from the JSON text into libdprf's list mode (dprf_amd.payload.parse_message ->
Context.verify_blob): no per-candidate Python, one library context per stream over this client's GPUs kept
across payloads (the library splits each payload over them).  "found" is the lowest list index
that verifies (the reference reports whichever of its 4 racing workers exits first).
"""
import argparse
import json
import socket
import sys
import textwrap
import threading
import time
import uuid

from . import _lib
from .brute_force import parse_verification_data
from .payload import candidate, parse_message

HEARTBEAT_PORT = 31337
HEARTBEAT_EVERY_S = 20


def recvall(connection, deadline=None):
    """Read until the peer half-closes.  deadline: time.time() limit; a peer still silent then raises
    socket.timeout (a socket with a timeout but no deadline keeps waiting, as the reference does)."""
    chunks = []
    while True:
        try:
            chunk = connection.recv(1 << 20)
        except socket.timeout:
            if deadline is not None and time.time() >= deadline:
                raise
            continue
        if not chunk:
            return b"".join(chunks)
        chunks.append(chunk)


def prepare_message(identifier, found, password, hearthbeat=False):
    """client.py:71-80"""
    data = {}
    if not hearthbeat:
        data["found"] = True if found else False
        data["correct_password"] = password if password else ""
    data["id"] = identifier
    return json.dumps(data).encode()


class GpuVerifier:
    """Verifies payloads on this client's GPUs through one library context over all of them (the library
    splits each payload into chunks over the devices); the context is created once per verifier stream."""

    def __init__(self, devices=None):
        if devices is None:
            devices = _lib.device_list()
            if not devices:
                raise _lib.DprfError(_lib.E_NODEVICE, "no gfx950 device visible")
        self.devices = list(devices)
        self.stream = None
        self.ctx = None
        self.verified = 0
        self.skipped = 0
        self.gpu_s = 0.0

    def _context(self, stream):
        if stream != self.stream:
            self.close()
            self.ctx = _lib.Context(parse_verification_data(stream), devices=self.devices)
            self.stream = stream
        return self.ctx

    def __call__(self, stream, blob, offsets):
        """(found, password) for one payload, found = the lowest list index that verifies.  A payload with
        candidates the reference cannot verify (NUL, empty or invalid-UTF-8 Office passwords, PDF R6 over 176
        bytes where the reference aborts, over an argv string's 131,071 bytes; include/dprf.h) is
        verified without them -- the reference fails such a candidate in its own verifier process and goes
        on with the rest (brute_force.py:106-161) -- instead of failing the payload on every client."""
        import numpy as np
        ctx = self._context(stream)
        n = len(offsets) - 1
        t0 = time.time()
        try:
            h, _, _ = ctx.verify_blob(blob, offsets, stop_on_first=True, cap=1)
            idx = h[0] if h else None
        except _lib.DprfError as e:
            if e.code not in (_lib.E_INVALID, _lib.E_DOMAIN, _lib.E_PWLEN):
                raise
            offs = np.asarray(offsets, dtype=np.uint64)
            keep = np.flatnonzero(ctx.list_status(blob, offs) == 0)
            self.skipped += n - len(keep)
            print("Skipping %d candidate(s) the verifier cannot take (%s)" % (n - len(keep), e), flush=True)
            idx = None
            if len(keep):
                buf = np.frombuffer(bytes(blob), dtype=np.uint8)
                parts = [buf[int(offs[k]):int(offs[k + 1])] for k in keep]
                sub = np.concatenate([np.zeros(1, np.uint64), np.cumsum([len(p) for p in parts], dtype=np.uint64)])
                h, _, _ = ctx.verify_blob(np.concatenate(parts).tobytes() if parts else b"", sub,
                                          stop_on_first=True, cap=1)
                idx = int(keep[h[0]]) if h else None
        self.gpu_s += time.time() - t0
        self.verified += n
        if idx is not None:
            return 1, candidate(blob, offsets, idx)
        return 0, None

    def close(self):
        if self.ctx is not None:
            self.ctx.close()
        self.ctx = None
        self.stream = None


class DryRun:
    """Stand-in verifier for protocol benchmarks: counts candidates, finds nothing, touches no GPU."""

    def __init__(self):
        self.verified = 0
        self.gpu_s = 0.0

    def __call__(self, stream, blob, offsets):
        self.verified += len(offsets) - 1
        return 0, None

    def close(self):
        pass


def connect_to_server(tcp_ip, tcp_port, identifier, verify, quiet=False):
    """client.py:36-69.  verify(stream, blob, offsets) -> (found, password)."""
    found, password = False, None
    while not found:
        try:
            client = socket.create_connection((tcp_ip, tcp_port))
            client.sendall(prepare_message(identifier, found, password))
            client.shutdown(socket.SHUT_WR)
            json_data = recvall(client)
            client.close()
        except OSError:
            print("Can't continue with brute-force. The server seems to be down.", flush=True)
            return 1, None
        if not json_data:
            if not quiet:
                print("No data received from server. Exiting.", flush=True)
            return 1, None
        if not quiet:
            print("Received data. Initializing brute-force...", flush=True)
        stream, blob, offsets = parse_message(json_data)
        if not stream:
            print("Empty data received from server.", flush=True)
            return 1, None
        if len(offsets) <= 1:
            print("No passwords provided by server.", flush=True)
            return 1, None
        found, password = verify(stream, blob, offsets)
        if not quiet:
            print("Finished brute-force attack. Sending the results to server.", flush=True)
    try:
        client = socket.create_connection((tcp_ip, tcp_port))
        client.sendall(prepare_message(identifier, found, password))
        client.shutdown(socket.SHUT_WR)
        client.close()
    except OSError:
        print("Failed to send found password to server (connection was refused).", flush=True)
    return 0, password


def hearthbeat(tcp_ip, identifier, port=HEARTBEAT_PORT, every=HEARTBEAT_EVERY_S, stop=None):
    """client.py:101-116"""
    stop = stop or threading.Event()
    while not stop.wait(every):
        try:
            client = socket.create_connection((tcp_ip, port), timeout=10)
            client.sendall(prepare_message(identifier, None, None, True))
            client.shutdown(socket.SHUT_WR)
            try:
                recvall(client, deadline=time.time() + 10)   # socket.timeout is an OSError: a failed beat
            finally:
                client.close()
        except OSError:
            print("Hearthbeat failed. Server seems to be down.", flush=True)
            return


def main(argv=None):
    parser = argparse.ArgumentParser(
        prog="DDPBFC",
        formatter_class=argparse.RawDescriptionHelpFormatter,
        description=textwrap.dedent("""\
            Distributed Document Password Brute-Force Framework Client (MI355X engine)
            """))
    parser.add_argument("tcp_ip", help="IP of the synchronization server")
    parser.add_argument("tcp_port", help="port on which synchronization server is listening")
    parser.add_argument("--devices", default=None, help="comma-separated GPU ordinals (default: all visible)")
    parser.add_argument("--heartbeat-port", type=int, default=HEARTBEAT_PORT)
    parser.add_argument("--quiet", action="store_true")
    parser.add_argument("--dry-run", action="store_true",
                        help="parse payloads but verify nothing (measures the server and the protocol alone)")
    args = parser.parse_args(argv)

    identifier = str(uuid.uuid4())
    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    verify = DryRun() if args.dry_run else GpuVerifier(devices)
    t = threading.Thread(target=hearthbeat, name="Hearthbeat", args=(args.tcp_ip, identifier, args.heartbeat_port),
                         daemon=True)
    t.start()
    t0 = time.time()
    rc, pw = connect_to_server(args.tcp_ip, int(args.tcp_port), identifier, verify, quiet=args.quiet)
    dt = time.time() - t0
    print(json.dumps({"client": identifier, "verified": verify.verified, "wall_s": dt, "gpu_s": verify.gpu_s,
                      "client_rate": verify.verified / max(dt, 1e-9),
                      "gpu_rate": verify.verified / max(verify.gpu_s, 1e-9), "password": pw}), flush=True)
    verify.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())

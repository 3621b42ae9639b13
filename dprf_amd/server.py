#!/usr/bin/env python3
"""Distributed Document Password Brute-Force Framework Server -- Python-3 counterpart of
/root/reference/src/server.py with the same CLI, TCP/JSON protocol and client bookkeeping:

* ``python -m dprf_amd.server document_type filename [-pr N] [-ps SIZE] tcp_ip tcp_port`` (server.py:310-329)
* work port: a client connects, sends ``{"found", "correct_password", "id"}`` and half-closes; the server
  answers ``{"data": stream, "passwords": [...]}`` or closes without data when the keyspace is exhausted
  (handle_connection :124-167); the first "found" ends the server (:114-119).
* heartbeat port 31337: ``{"id"}`` refreshes the client, the answer is ``{"found": ...}`` (:209-238);
  clients silent for 120 s are dropped every 120 s and their outstanding payload is re-queued (:241-256).
* candidates: lengths 1..N (default 8) of ``string.lowercase`` in ``itertools.product`` order (:189-199).

Differences, all below the protocol: the candidate source is a global keyspace index instead of a
generator process feeding a ``JoinableQueue`` one password at a time, and payload JSON is produced by
numpy (dprf_amd.payload) -- the reference's ceiling is ~10^5 candidates/s, one MI355X client verifies
10^6..10^9/s depending on the format.  Outstanding payloads are remembered as index segments.
Extensions: ``--charset``, ``--heartbeat-port`` (so that several servers can share a host) and
``--max-candidates`` (a bounded run for benchmarks).
"""
import argparse
import collections
import concurrent.futures
import json
import socket
import sys
import textwrap
import threading
import time
from datetime import datetime, timedelta

from .payload import LOWERCASE, Keyspace, build_message

HEARTBEAT_PORT = 31337
INACTIVE_AFTER_S = 120          # server.py:52-53
CLEANUP_EVERY_S = 120           # server.py:241-244
REQUEST_TIMEOUT_S = 60          # a work request not finished in this time is dropped (reference: waits forever)


class Client:
    """A brute-force client connected to the server (server.py:39-58)."""

    def __init__(self, id, last_activity):
        self.id = id
        self.last_activity = last_activity

    def __str__(self):
        return "ID: " + self.id + " Last activity: " + str(self.last_activity)

    def __eq__(self, other):
        return self.id == other.id

    def isActive(self, now=None, inactive_after=INACTIVE_AFTER_S):
        now = now or datetime.now()
        return self.last_activity > now - timedelta(seconds=inactive_after)

    def refresh(self, last_activity):
        self.last_activity = last_activity


def recvall(connection, deadline=None):
    """Read until the peer half-closes (server.py:171-183).  deadline: time.time() limit after which a peer
    that is still silent raises socket.timeout (an OSError) instead of holding the thread forever."""
    chunks = []
    while True:
        try:
            chunk = connection.recv(1 << 16)
        except socket.timeout:
            if deadline is not None and time.time() >= deadline:
                raise
            continue
        if not chunk:
            return b"".join(chunks)
        chunks.append(chunk)


class Server:
    """State and threads of one server run (run_server, server.py:61-121)."""

    def __init__(self, stream, password_range=None, payload_size=20000, charset=LOWERCASE,
                 heartbeat_port=HEARTBEAT_PORT, max_candidates=None, inactive_after=INACTIVE_AFTER_S,
                 cleanup_every=CLEANUP_EVERY_S, quiet=False, builders=4, depth=6):
        self.stream = stream
        self.payload_size = int(payload_size)
        self.charset = charset
        self.keyspace = Keyspace(charset, password_range if password_range else 8, limit=max_candidates)
        self.heartbeat_port = heartbeat_port
        self.inactive_after = inactive_after
        self.cleanup_every = cleanup_every
        self.quiet = quiet
        self.clients = []
        self.processed_passwords = {}     # client id -> segments of its outstanding payload
        self.requeue = collections.deque()
        self.cursor = 0
        self.counter = 0
        self.found = False
        self.correct_password = None
        self.lock = threading.Lock()
        self.stop = threading.Event()
        self.bound = threading.Event()
        self.address = None
        self.first_send = None
        self.pool = concurrent.futures.ThreadPoolExecutor(max_workers=max(1, builders))
        self.depth = max(1, depth)
        self.pending = collections.deque()     # futures of prebuilt payloads, in keyspace order

    def log(self, *a):
        if not self.quiet:
            print(*a, flush=True)

    # -- candidate source (generate + get_passwords, server.py:186-307) -----------------------------
    def take_segments(self):
        with self.lock:
            if self.requeue:
                return self.requeue.popleft()
            segs = self.keyspace.segments(self.cursor, self.payload_size)
            self.cursor += sum(c for _, _, c in segs)
            return segs

    def prepare_data_for_transfer(self):
        """Next payload (message bytes, segments) or (None, None) when nothing is left to hand out.
        Payloads are built ahead by a small thread pool (numpy releases the GIL), in keyspace order,
        so building overlaps the socket work of the accept loop."""
        with self.lock:
            if self.requeue:              # an inactive client's payload goes out first, rebuilt
                segs = self.requeue.popleft()
                return build_message(self.stream, self.charset, segs), segs
        while len(self.pending) < self.depth:
            segs = self.take_segments()
            if not segs:
                break
            self.pending.append(self.pool.submit(lambda sg=segs: (build_message(self.stream, self.charset, sg), sg)))
        if not self.pending:
            return None, None
        return self.pending.popleft().result()

    # -- work port ----------------------------------------------------------------------------------
    def handle_connection(self, client, address, message, segs):
        found = False
        self.log("A client connected from address:", address)
        try:
            client.settimeout(REQUEST_TIMEOUT_S)
            data = json.loads(recvall(client, deadline=time.time() + REQUEST_TIMEOUT_S))
            client.shutdown(socket.SHUT_RD)
            client_identifier = data["id"]
        except (OSError, ValueError, KeyError, TypeError):
            client.close()                   # not a client message (e.g. a port probe): ignore it
            return False, False
        sent = False
        with self.lock:
            known = client_identifier in (x.id for x in self.clients)
            if not known:
                if message:
                    self.clients.append(Client(client_identifier, datetime.now()))
                else:
                    client.close()
                    return False, False
            else:
                # a known client coming back has finished its previous chunk (server.py:142-145)
                done = self.processed_passwords.pop(client_identifier, None)
                self.counter += sum(c for _, _, c in done) if done else self.payload_size
        if data.get("found"):
            self.log("Correct password is: ", data.get("correct_password"))
            self.correct_password = data.get("correct_password")
            found = True
        elif message:
            try:
                client.sendall(message)
            except OSError:
                # the client died between its request and our answer: keep the payload for the next
                # connection (the caller still holds message/segs) and forget a client that never got one
                client.close()
                if not known:
                    with self.lock:
                        self.clients = [c for c in self.clients if c.id != client_identifier]
                return False, False
            if self.first_send is None:
                self.first_send = time.time()
            with self.lock:
                self.processed_passwords[client_identifier] = segs
            sent = True
            self.log("Sent new instruction to: ", address)
        else:
            with self.lock:
                self.clients = [c for c in self.clients if c.id != client_identifier]
        client.close()
        return found, sent

    # -- heartbeat port (server.py:209-238) ----------------------------------------------------------
    def heartbeat(self, tcp_ip):
        try:
            server = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            server.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            server.bind((tcp_ip, self.heartbeat_port))
            server.listen(64)
            server.settimeout(0.5)
        except OSError as ex:
            self.log("Error opening heartbeat socket:", ex)
            return
        while not self.stop.is_set():
            try:
                client, address = server.accept()
            except socket.timeout:
                continue
            except OSError:
                break
            try:
                client.settimeout(10)
                data = json.loads(recvall(client, deadline=time.time() + 10))
                with self.lock:
                    for c in self.clients:
                        if c.id == data.get("id"):
                            c.refresh(datetime.now())
                client.sendall(json.dumps({"found": bool(self.found)}).encode())
            except (OSError, ValueError):
                pass
            finally:
                client.close()
        server.close()

    # -- inactive clients (server.py:241-256) --------------------------------------------------------
    def remove_inactive_clients(self):
        while not self.stop.wait(self.cleanup_every):
            with self.lock:
                now = datetime.now()
                inactive = [c for c in self.clients if not c.isActive(now, self.inactive_after)]
                for c in inactive:
                    self.log("Client ", c.id, " is inactive.")
                    self.clients.remove(c)
                    segs = self.processed_passwords.pop(c.id, None)
                    if segs:
                        self.requeue.append(segs)
                    self.log("Active clients: ", len(self.clients))

    def run(self, tcp_ip, tcp_port):
        threading.Thread(target=self.heartbeat, name="Hearthbeat", args=(tcp_ip,), daemon=True).start()
        threading.Thread(target=self.remove_inactive_clients, name="Client clean-up", daemon=True).start()
        try:
            server = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            server.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            server.bind((tcp_ip, tcp_port))
            server.listen(64)
        except OSError as ex:
            self.log("Error opening socket:", ex)
            self.stop.set()
            return None
        self.address = server.getsockname()
        self.bound.set()
        start_time = time.time()
        message, segs = None, None
        try:
            while not self.stop.is_set():
                self.log("Number of clients: " + str(len(self.clients)))
                self.log("Estimated speed: " + str(self.counter / max(time.time() - start_time, 1e-9)) + " H/sec")
                if message is None:
                    message, segs = self.prepare_data_for_transfer()
                if not message and not self.clients:
                    self.log("Password is not in brute-forced space.")
                    return None
                client, address = server.accept()
                if not message:
                    message, segs = self.prepare_data_for_transfer()
                result, sent = self.handle_connection(client, address, message, segs)
                if sent:
                    message, segs = None, None
                if result:
                    self.found = True
                    return self.correct_password
        except KeyboardInterrupt:
            self.log("Stoping server...")
            return None
        finally:
            self.end_time = time.time()
            self.elapsed = self.end_time - start_time
            self.stop.set()
            self.pool.shutdown(wait=False, cancel_futures=True)
            server.close()


def get_verification_data(doc_type, filename):
    """Parse the document (server.py:310-321); ODF uses the full (non -e) stream like the reference
    server (:316), unlike brute_force.py's -e (:239)."""
    print("Parsing " + filename + "...")
    if doc_type == '1':
        from .parsers import office2john
        return office2john.get_hash(filename).strip()
    if doc_type == '2':
        from .parsers import odt2hashes
        return odt2hashes.get_hashes(filename, experimental=False).strip()
    if doc_type == '3':
        from .parsers import pdf2john
        return pdf2john.get_hash(filename).strip()


def main(argv=None):
    parser = argparse.ArgumentParser(
        prog="DDPBFS",
        formatter_class=argparse.RawDescriptionHelpFormatter,
        description=textwrap.dedent("""\
            Distributed Document Password Brute-Force Framework Server (MI355X engine)

            Document types:
                1: Microsoft Office
                2: OpenDocument
                3: Portable Document Format
            """))
    parser.add_argument("document_type", help="type of the protected document (MS Office / OpenDocument)")
    parser.add_argument("filename", help="the protected document")
    parser.add_argument("-pr", "--passwordrange", type=int, help="password range to brute-force (i.e., 2 -> aa..zz, default 8)")
    parser.add_argument("-ps", "--payloadsize", type=int, help="number of passwords sent to clients (default 20000)")
    parser.add_argument("tcp_ip", help="IP address to which clients should connect")
    parser.add_argument("tcp_port", help="port to which clients should connect")
    parser.add_argument("--charset", default=LOWERCASE, help="candidate alphabet (default a-z)")
    parser.add_argument("--heartbeat-port", type=int, default=HEARTBEAT_PORT)
    parser.add_argument("--max-candidates", type=int, default=None, help="stop after this many candidates")
    parser.add_argument("--stream", default=None, help="verifier stream instead of parsing filename")
    parser.add_argument("--builders", type=int, default=4, help="payload builder threads")
    parser.add_argument("--quiet", action="store_true")
    args = parser.parse_args(argv)

    stream = args.stream or get_verification_data(args.document_type, args.filename)
    if not stream:
        sys.exit(0)
    srv = Server(stream, args.passwordrange, args.payloadsize if args.payloadsize else 20000, args.charset,
                 args.heartbeat_port, args.max_candidates, quiet=args.quiet, builders=args.builders)
    pw = srv.run(args.tcp_ip, int(args.tcp_port))
    n = srv.counter
    busy = srv.end_time - (srv.first_send or srv.end_time)
    print(json.dumps({"server": "done", "acknowledged": n, "elapsed_s": srv.elapsed, "from_first_payload_s": busy,
                      "rate": n / max(busy, 1e-9), "password": pw}), flush=True)
    return pw


if __name__ == "__main__":
    main()

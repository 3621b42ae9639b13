#!/usr/bin/env python3
"""Document Password Brute-Forcer on MI355X -- Python-3 counterpart of /root/reference/src/brute_force.py.

Same module surface, same names, same argument meaning and return values:

* ``init(stream, password_range, passwords) -> (found, password)`` (brute_force.py:39-57): exactly one of
  a range length or a candidate list; ``found`` is 0/1 and ``password`` is the literal
  ``"default_password_allocation"`` when nothing is found (:64, :79).
* ``init_rangebased_brute_force`` (:60-79): every ``charset^N`` candidate in ``itertools.product`` order
  (:205) plus the literal ``"_dummy"`` the reference also queues (:76).
* ``init_listbased_brute_force`` (:82-104): the explicit list a ``client.py`` payload carries (client.py:105).
* ``get_verification_data`` / ``parse_verification_data`` (:232-264) and the CLI (:266-298).

What changes is underneath: instead of one ``Popen`` of an OpenSSL verifier per candidate (:163-197) the
candidates go to libdprf.so in batches, one candidate per GPU lane.  Differences, all deliberate:

* "found" is the LOWEST keyspace index that verifies (``_dummy`` first), not whichever of four racing
  workers exits first.
* a verifier error is raised as :class:`dprf_amd._lib.DprfError`, never reported as found (the reference
  counts any non-zero exit as a hit, :140; Appendix B.6).
* optional keyword arguments ``charset`` (default lowercase a-z, Python 2 ``string.lowercase`` in the C
  locale), ``devices`` (default: every visible gfx950 GPU) and ``checkpoint`` (a resumable cursor file
  for range mode, :class:`Checkpoint`).
"""
import argparse
import re
import sys
import textwrap
import threading
import time

from . import _lib

LOWERCASE = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWERCASE + LOWERCASE.upper() + "0123456789"   # the configs' "alnum" order: a-z A-Z 0-9
DEFAULT_PASSWORD = "default_password_allocation"
DUMMY = "_dummy"
ROUND_PER_DEVICE = 1 << 24      # candidates per device between stop checks in range mode


def init(stream, password_range, passwords, charset=LOWERCASE, devices=None, checkpoint=None):
    # The common entry point (brute_force.py:39-57)
    if not password_range and not passwords:
        raise ValueError('Need to provide a password range to generate or a list of passwords.')
    if password_range and passwords:
        raise ValueError('Need to provide either a password range or a password list (not both).')

    input_data = parse_verification_data(stream)
    print("Initializing brute-force.")

    try:
        if password_range and not passwords:
            return init_rangebased_brute_force(input_data, password_range, charset=charset, devices=devices,
                                               checkpoint=checkpoint)
        if passwords and not password_range:
            return init_listbased_brute_force(input_data, passwords, devices=devices)
    except KeyboardInterrupt:
        sys.exit(0)


def _devices(devices):
    if devices is None:
        n = _lib.device_count()
        if n < 1:
            raise _lib.DprfError(_lib.E_NODEVICE, "no gfx950 device visible")
        return list(range(n))
    return list(devices)


def _contexts(input_data, devices):
    return [_lib.Context(input_data, device=d) for d in _devices(devices)]


def _report(found_pw, n, t0):
    dt = max(time.time() - t0, 1e-9)
    print("Tried %d candidates in %.3f s (%.0f H/sec)" % (n, dt, n / dt))
    if found_pw is not None:
        print("Correct password is '" + found_pw + "'")


class Checkpoint:
    """Resumable shard cursor for range mode (an extension; the reference has none).  A JSON file records
    which search it belongs to (SHA-256 of the verifier stream, charset, length) and the keyspace index
    below which every candidate has been verified; it is rewritten atomically after every round, so an
    interrupted run restarts at its last completed round."""

    def __init__(self, path, input_data, charset, pwlen):
        import hashlib
        self.path = path
        self.key = {"stream_sha256": hashlib.sha256("*".join(map(str, input_data)).encode()).hexdigest(),
                    "charset": charset, "pwlen": int(pwlen)}

    def load(self):
        """(next index, found password or None) recorded for this search; (0, None) when there is none."""
        import json
        import os
        if not self.path or not os.path.exists(self.path):
            return 0, None
        with open(self.path) as f:
            d = json.load(f)
        if any(d.get(k) != v for k, v in self.key.items()):
            raise ValueError("checkpoint %s belongs to a different search" % self.path)
        return int(d["next_index"]), d.get("found")

    def save(self, next_index, found=None):
        import json
        import os
        if not self.path:
            return
        tmp = self.path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(dict(self.key, next_index=int(next_index), found=found), f)
        os.replace(tmp, self.path)


def init_rangebased_brute_force(input_data, password_range, charset=LOWERCASE, devices=None, checkpoint=None):
    """charset^password_range in product order, plus "_dummy" (brute_force.py:60-79, :199-219).

    Multi-GPU: each round gives every device a contiguous slice of one contiguous block of the keyspace,
    so after a round every index below the round's end has been verified and the lowest hit of the
    first round that has one is the lowest hit overall.  checkpoint: path of a resumable cursor file
    (:class:`Checkpoint`)."""
    cp = Checkpoint(checkpoint, input_data, charset, password_range)
    done, prior = cp.load()
    if prior is not None:
        print("Checkpoint: search already finished, password '%s'" % prior)
        return 1, prior
    ctxs = _contexts(input_data, devices)
    t0 = time.time()
    try:
        if done == 0:
            hits, _, _ = ctxs[0].verify_list([DUMMY], stop_on_first=True, cap=1)
            if hits:
                cp.save(0, DUMMY)
                _report(DUMMY, 1, t0)
                return 1, DUMMY
        else:
            print("Checkpoint: resuming at index %d" % done)
        space = len(charset) ** password_range
        found = None
        while done < space and found is None:
            block = min(space - done, ROUND_PER_DEVICE * len(ctxs))
            slices = _round_slices(done, block, len(ctxs))
            results = [None] * len(ctxs)

            def work(k):
                s, n = slices[k]
                results[k] = ctxs[k].search_range(charset, password_range, s, n, stop_on_first=True, cap=1) if n else ([], 0, {})

            if len(ctxs) == 1:
                work(0)
            else:
                ths = [threading.Thread(target=work, args=(k,)) for k in range(len(ctxs))]
                [t.start() for t in ths]
                [t.join() for t in ths]
            firsts = [r[0][0] for r in results if r[0]]
            if firsts:
                idx = min(firsts)
                found = _index_to_password(idx, charset, password_range)
            done += block
            cp.save(done, found)
        _report(found, done + 1, t0)
        return (1, found) if found is not None else (0, DEFAULT_PASSWORD)
    finally:
        for c in ctxs:
            c.close()


def _round_slices(done, block, ndev):
    """Contiguous (start, count) slices, one per device, tiling [done, done + block)."""
    per = -(-block // ndev)
    out = []
    for k in range(ndev):
        s = done + k * per
        out.append((min(s, done + block), max(0, min(per, done + block - s))))
    return out


def init_listbased_brute_force(input_data, passwords, devices=None):
    """An explicit candidate list, e.g. a server payload (brute_force.py:82-104).  The list is split
    into contiguous slices, one per device; the lowest-index hit wins."""
    passwords = list(passwords)
    ctxs = _contexts(input_data, devices)
    t0 = time.time()
    try:
        per = -(-len(passwords) // len(ctxs))
        results = [None] * len(ctxs)

        def work(k):
            sl = passwords[k * per:(k + 1) * per]
            results[k] = ctxs[k].verify_list(sl, stop_on_first=True, cap=1) if sl else ([], 0, {})

        if len(ctxs) == 1:
            work(0)
        else:
            ths = [threading.Thread(target=work, args=(k,)) for k in range(len(ctxs))]
            [t.start() for t in ths]
            [t.join() for t in ths]
        found = None
        for k, r in enumerate(results):
            if r[0]:
                found = passwords[k * per + r[0][0]]
                break
        _report(found, len(passwords), t0)
        return (1, found) if found is not None else (0, DEFAULT_PASSWORD)
    finally:
        for c in ctxs:
            c.close()


def _index_to_password(idx, charset, n):
    out = []
    for _ in range(n):
        out.append(charset[idx % len(charset)])
        idx //= len(charset)
    return "".join(reversed(out))


def get_verification_data(doc_type, filename):
    """Parse the document into the verifier stream (brute_force.py:232-242).  ODF uses the -e
    (experimental, smallest encrypted file) data exactly like the reference engine (:239)."""
    print("Parsing " + filename + "...")
    if doc_type == '1':
        from .parsers import office2john
        return office2john.get_hash(filename).strip()
    if doc_type == '2':
        from .parsers import odt2hashes
        return odt2hashes.get_hashes(filename, experimental=True).strip()
    if doc_type == '3':
        from .parsers import pdf2john
        return pdf2john.get_hash(filename).strip()


def parse_verification_data(stream):
    """Field split + format tag (brute_force.py:245-264), verbatim semantics."""
    print("Preparing verification data...")
    data_array = re.split(r"(?:\*)", stream)
    m = re.search(r".*:\$(\w+)\$", data_array[0])
    data_format = m.groups()[0] if m else None
    data_array[0] = data_format
    if data_format == "office" and len(data_array) == 8:
        return data_array
    if data_format == "odt" and len(data_array) == 7:
        return data_array
    if data_format == "pdf" and len(data_array) == 12:
        return data_array
    print("The input data is not supported.")
    sys.exit(1)


def main(argv=None):
    parser = argparse.ArgumentParser(
        prog="DPBF",
        formatter_class=argparse.RawDescriptionHelpFormatter,
        description=textwrap.dedent("""\
            Document Password Brute-Forcer (MI355X engine)

            Document types:
                1: Microsoft Office
                2: OpenDocument
                3: Portable Document Format

            Actually supported formats:
                Office Document Structure - EncryptionInfo Stream (Standard Encryption) (Office 2007)
                OpenDocument - v1.2 with AES-256 in CBC mode
                Portable Document Format - PDF 1.3 - 1.7 (Standard Security Handlers v1-5 r2-6)
            """))
    parser.add_argument("document_type", help="type of the protected document")
    parser.add_argument("filename", help="the protected document")
    parser.add_argument("-pr", "--passwordrange", type=int, help="password range to brute-force (i.e., 2 -> aa..zz)")
    parser.add_argument("--charset", default=LOWERCASE, help="candidate alphabet (default a-z)")
    parser.add_argument("--devices", default=None, help="comma-separated GPU ordinals (default: all)")
    parser.add_argument("--checkpoint", default=None, help="resumable cursor file (written after every round)")
    args = parser.parse_args(argv)

    stream = get_verification_data(args.document_type, args.filename)
    if not stream:
        sys.exit(0)
    devices = [int(x) for x in args.devices.split(",")] if args.devices else None
    found, password = init(stream, args.passwordrange if args.passwordrange else 8, None,
                           charset=args.charset, devices=devices, checkpoint=args.checkpoint)
    if not found:
        print("Password is not in brute-forced space.")
    return found, password


if __name__ == "__main__":
    main()

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
  locale; distinct characters, any of them non-ASCII too -- :func:`check_charset`), ``devices`` (default:
  every visible gfx950 GPU) and ``checkpoint`` (a resumable cursor file for range mode, :class:`Checkpoint`).

The reference's four worker processes on one queue (:70-73, :92-95) are inside libdprf.so: one context
spans the devices, and every search call fans out over them (one worker thread + HIP stream per GPU on a
shared chunk cursor, include/dprf.h).  Range mode calls it in rounds of about ROUND_SECONDS of work so the
checkpoint cursor advances and Ctrl-C is honoured between rounds.
"""
import argparse
import re
import sys
import textwrap
import time

from . import _lib

LOWERCASE = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWERCASE + LOWERCASE.upper() + "0123456789"   # the configs' "alnum" order: a-z A-Z 0-9
DEFAULT_PASSWORD = "default_password_allocation"
DUMMY = "_dummy"
ROUND_SECONDS = 5.0              # range mode: wall time of one library call (checkpoint / Ctrl-C granularity)
FIRST_ROUND = 1 << 22           # least candidates of the first round, before a rate is known
ROUND_CHUNKS = 4                 # a round lasts at least this many of the library's largest chunks (0: fixed
                                 # FIRST_ROUND / ROUND_SECONDS only)
ROUND_MAX_SECONDS = 12.0         # ... but never longer (R6's 2^25-candidate chunks, ~9 s each, would make
                                 # multi-GPU rounds ~36 s -- the checkpoint / Ctrl-C granularity; the guided split of
                                 # dprf_plan_chunk sizes the chunks of a shorter round down by itself)
_HUGE = 1 << 62


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
        devs = _lib.device_list()
        if not devs:
            raise _lib.DprfError(_lib.E_NODEVICE, "no gfx950 device visible")
        return devs
    return list(devices)


def _context(input_data, devices):
    """One library context over the devices (the library splits every call over them)."""
    return _lib.Context(input_data, devices=_devices(devices))


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


def first_round(kernel, ndev):
    """Candidates of the first range-mode round: ROUND_CHUNKS first chunks per device (the library's policy before
    a rate is measured, dprf_plan_chunk), so no device idles in round 1 and its guided tail stays short.  One device
    has no guided tail: its rounds stay at FIRST_ROUND / ROUND_SECONDS, the checkpoint and Ctrl-C granularity
    (ADVICE r3)."""
    if not ROUND_CHUNKS or kernel is None or ndev <= 1:
        return FIRST_ROUND
    return max(FIRST_ROUND, ROUND_CHUNKS * ndev * _lib.plan_chunk(kernel, 0.0, _HUGE, _HUGE, 1))


def round_seconds(kernel, rate, ndev):
    """Wall time of one round at `rate` (cand/s over all devices): ROUND_SECONDS, or ROUND_CHUNKS times the
    library's largest chunk at the per-device rate if that is longer, so the guided tail of a call (chunks
    shrinking to the family's floor, include/dprf.h dprf_plan_chunk) stays a small part of the round."""
    per_dev_ms = rate / 1e3 / max(1, ndev)
    if per_dev_ms <= 0 or not ROUND_CHUNKS or kernel is None or ndev <= 1:
        return ROUND_SECONDS
    big = _lib.plan_chunk(kernel, per_dev_ms, _HUGE, _HUGE, 1)
    return min(ROUND_MAX_SECONDS, max(ROUND_SECONDS, ROUND_CHUNKS * big / per_dev_ms / 1e3))


def next_round(rate, remaining, seconds=ROUND_SECONDS, first=FIRST_ROUND):
    """Candidates of the next range-mode round: ~`seconds` at the measured rate (cand/s; 0 = unknown)."""
    n = first if rate <= 0 else max(first, int(rate * seconds))
    return min(remaining, n)


def progress(t0, tried, remaining):
    """The reference's progress report (brute_force.py:149-157: every 1000 candidates there, every round here):
    running time, candidates tried, speed, and what is left to verify (the reference's queue size)."""
    actual = time.time()
    speed = tried / max(actual - t0, 1e-9)
    print("Running time: " + str(actual - t0) + " & tried since: " + str(tried) + " passes")
    print("Speed: " + str(speed) + " H/sec")
    print("Queue size: " + str(remaining))
    sys.stdout.flush()


def check_charset(charset):
    """The range-mode alphabet: a non-empty str of distinct characters without NUL (NUL cannot reach the reference's
    verifier through argv).  Returns True when every character is one byte (ASCII) -- the library enumerates such a
    charset on the device (dprf_search_range) -- and False when some character takes more UTF-8 bytes: the library's
    range symbols are bytes, so such a window is spelled on the host by characters (payload.spell_utf8) and verified in
    list mode (dprf_verify_list), the keyspace staying charset^N over characters as itertools.product has it
    (brute_force.py:199-219).  Raises DprfError(E_CHARSET) otherwise."""
    if not isinstance(charset, str):
        raise _lib.DprfError(_lib.E_CHARSET, "charset must be a str (got %s)" % type(charset).__name__)
    if not charset:
        raise _lib.DprfError(_lib.E_CHARSET, "empty charset")
    if "\0" in charset:
        raise _lib.DprfError(_lib.E_CHARSET, "charset contains NUL (the reference passes candidates via argv)")
    if len(set(charset)) != len(charset):
        dup = next(c for c in charset if charset.count(c) > 1)
        raise _lib.DprfError(_lib.E_CHARSET, "charset repeats %r (itertools.product would verify candidates twice)"
                             % dup)
    try:
        charset.encode("utf-8")
    except UnicodeEncodeError as e:   # lone surrogates
        raise _lib.DprfError(_lib.E_CHARSET, "charset is not encodable as UTF-8: %s" % e)
    return all(ord(c) < 0x80 for c in charset)


WIDE_ROUND = 1 << 21   # candidates per library call of a host-spelled (non-ASCII charset) round


def search_round(ctx, charset, pwlen, start, count, stop_on_first=True):
    """One round of range mode on every device of ctx: (lowest hit index or None, stats).  The same call
    bench.py times per rank (there with stop_on_first=False: a throughput step verifies its whole batch
    even when a false positive of ODF -e's 2-byte check turns up in it).  A charset with multi-byte characters
    (check_charset False) is enumerated by character: spelled on the device (ctx.search_symbols, ABI 7) when every
    candidate fits a 64-byte list slot, else spelled on the host and verified as a list, in calls of WIDE_ROUND
    candidates."""
    if check_charset(charset):
        hits, _, st = ctx.search_range(charset, pwlen, start, count, stop_on_first=stop_on_first, cap=1)
        return (hits[0] if hits else None), st
    if hasattr(ctx, "search_symbols"):
        try:
            hits, _, st = ctx.search_symbols(charset, pwlen, start, count, stop_on_first=stop_on_first, cap=1)
            return (hits[0] if hits else None), st
        except _lib.DprfError as ex:
            if ex.code != _lib.E_PWLEN:
                raise
    import os
    from .payload import spell_utf8_parallel
    total = {"candidates": 0, "wall_ms": 0.0}
    found = None
    workers = min(16, os.cpu_count() or 1)
    for s in range(start, start + count, WIDE_ROUND):
        n = min(WIDE_ROUND, start + count - s)
        blob, offs = spell_utf8_parallel(charset, pwlen, s, n, workers)
        hits, _, st = ctx.verify_blob(blob, offs, stop_on_first=stop_on_first, cap=1)
        total["candidates"] += st["candidates"]
        total["wall_ms"] += st["wall_ms"]
        if hits and found is None:
            found = s + hits[0]
            if stop_on_first:
                break
    return found, total


def init_rangebased_brute_force(input_data, password_range, charset=LOWERCASE, devices=None, checkpoint=None):
    """charset^password_range in product order, plus "_dummy" (brute_force.py:60-79, :199-219).

    Rounds of consecutive indices, each one library call over all devices with stop_on_first: a round
    returns its lowest hit, every index below a round's end has been verified once it returns, so the first
    round with a hit holds the lowest hit overall.  checkpoint: path of a resumable cursor file
    (:class:`Checkpoint`).  charset: see check_charset (raises before any device work)."""
    check_charset(charset)
    cp = Checkpoint(checkpoint, input_data, charset, password_range)
    done, prior = cp.load()
    if prior is not None:
        print("Checkpoint: search already finished, password '%s'" % prior)
        return 1, prior
    ctx = _context(input_data, devices)
    t0 = time.time()
    tried = 0
    try:
        if done == 0:
            hits, _, _ = ctx.verify_list([DUMMY], stop_on_first=True, cap=1)
            tried += 1
            if hits:
                cp.save(0, DUMMY)
                _report(DUMMY, tried, t0)
                return 1, DUMMY
        else:
            print("Checkpoint: resuming at index %d" % done)
        space = len(charset) ** password_range
        found, rate = None, 0.0
        ndev = len(getattr(ctx, "devices", [0]))
        kernel = getattr(ctx, "kernel", None)
        first = first_round(kernel, ndev)
        while done < space and found is None:
            n = next_round(rate, space - done, round_seconds(kernel, rate, ndev), first)
            idx, st = search_round(ctx, charset, password_range, done, n)
            tried += st["candidates"]
            rate = st["candidates"] / max(st["wall_ms"] / 1e3, 1e-9)
            if idx is not None:
                found = _index_to_password(idx, charset, password_range)
            done += n
            cp.save(done, found)
            progress(t0, tried, space - done if found is None else 0)
        _report(found, tried, t0)
        return (1, found) if found is not None else (0, DEFAULT_PASSWORD)
    finally:
        ctx.close()


def init_listbased_brute_force(input_data, passwords, devices=None):
    """An explicit candidate list, e.g. a server payload (brute_force.py:82-104): one library call over all
    devices; the lowest list index that verifies wins."""
    passwords = list(passwords)
    ctx = _context(input_data, devices)
    t0 = time.time()
    try:
        hits, _, _ = ctx.verify_list(passwords, stop_on_first=True, cap=1)
        found = passwords[hits[0]] if hits else None
        _report(found, len(passwords), t0)
        return (1, found) if found is not None else (0, DEFAULT_PASSWORD)
    finally:
        ctx.close()


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

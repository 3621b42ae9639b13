"""Server payloads of the reference's work-distribution protocol, built and parsed without per-candidate
Python work.

Wire format (unchanged, so reference clients and servers interoperate with these):
  server -> client  ``{"data": "<verifier stream>", "passwords": ["aaaa", "aaab", ...]}``
                    (server.py:285-292 ``prepare_data_for_transfer``; client.py:55 ``json.loads``)
  client -> server  ``{"found": bool, "correct_password": str, "id": uuid}`` (client.py:71-80)

The reference server enumerates lengths 1..N of ``string.lowercase`` in ``itertools.product`` order
(server.py:189-199) and hands out ``payload_size`` of them per message (server.py:294-307) through a
``JoinableQueue`` one ``put``/``get`` per password -- ~10^5 candidates/s, far below what one GPU
verifies.  Here the keyspace is addressed by a global index (:class:`Keyspace`), a payload is a list of
``(length, start, count)`` segments, and its JSON text is produced by numpy from the indices
(:func:`build_message`).  The GPU client parses the same JSON straight into the (blob, offsets) form
``dprf_verify_list`` takes (:func:`parse_message`), falling back to ``json.loads`` whenever the text
holds an escape sequence.
"""
import json

import numpy as np

LOWERCASE = "abcdefghijklmnopqrstuvwxyz"


class Keyspace:
    """charset^1 .. charset^max_len concatenated, each length in itertools.product order (leftmost
    character most significant) -- the order of server.py:189-199 (default lengths 1..8)."""

    def __init__(self, charset=LOWERCASE, max_len=8, limit=None):
        if not charset or len(set(charset)) != len(charset):
            raise ValueError("charset must be non-empty and without repeats")
        self.charset = charset
        self.max_len = int(max_len)
        self.sizes = [len(charset) ** L for L in range(1, self.max_len + 1)]
        self.total = sum(self.sizes)
        if limit is not None:
            self.total = min(self.total, int(limit))

    def segments(self, g0, n):
        """[(length, start_within_length, count)] covering global indices [g0, min(g0+n, total))."""
        out = []
        g, end = int(g0), min(int(g0) + int(n), self.total)
        base = 0
        for L, size in zip(range(1, self.max_len + 1), self.sizes):
            if g >= end:
                break
            if g < base + size:
                s = g - base
                c = min(size - s, end - g)
                out.append((L, s, c))
                g += c
            base += size
        return out

    def password(self, length, index):
        cs, out = self.charset, []
        for _ in range(length):
            out.append(cs[index % len(cs)])
            index //= len(cs)
        return "".join(reversed(out))

    def global_index(self, password):
        """Inverse of the enumeration (for tests and reporting)."""
        L = len(password)
        idx = 0
        for ch in password:
            idx = idx * len(self.charset) + self.charset.index(ch)
        return sum(self.sizes[:L - 1]) + idx


def _json_safe(charset):
    return all(0x20 <= ord(c) < 0x7f and c not in '"\\' for c in charset)


_TABLES = {}


def _chunk_table(charset):
    """(c, uint8[n^c, c]): every c-character string of the charset in product order, c chosen so that
    the table stays <= ~1 Mi rows; candidates are spelled by gathering c characters at a time."""
    t = _TABLES.get(charset)
    if t is None:
        n = len(charset)
        c = 1
        while n ** (c + 1) <= (1 << 20):
            c += 1
        cs = np.frombuffer(charset.encode("ascii"), dtype=np.uint8)
        idx = np.arange(n ** c, dtype=np.int64)
        tab = np.empty((n ** c, c), dtype=np.uint8)
        for p in range(c - 1, -1, -1):
            tab[:, p] = cs[idx % n]
            idx //= n
        t = _TABLES[charset] = (c, tab)
    return t


def segment_chars(charset, length, start, count, out=None):
    """uint8[count, length]: the candidates of one segment, spelled from their indices (written into
    `out` when given, e.g. a column slice of the JSON row array)."""
    n = len(charset)
    c, tab = _chunk_table(charset)
    if out is None:
        out = np.empty((count, length), dtype=np.uint8)
    idx = np.arange(start, start + count, dtype=np.int64)
    pos = length
    while pos > 0:
        w = min(c, pos)
        part = idx % (n ** w)
        idx //= n ** w
        out[:, pos - w:pos] = tab[part, c - w:] if w == c else tab[part * 1, c - w:]
        pos -= w
    return out


def spell_utf8(charset, length, start, count):
    """(blob, offsets) of keyspace indices [start, start+count) of charset^length in itertools.product order, each
    candidate the UTF-8 encoding of its characters: the dprf_verify_list form of a range window whose symbols are not
    all single bytes (range mode over a non-ASCII charset, brute_force.search_round).  A character is one symbol
    whatever its UTF-8 length, as in ``itertools.product(charset, repeat=length)``.  Vectorised per (position, byte):
    every candidate's bytes are scattered straight to their offsets (no per-candidate Python)."""
    syms = [c.encode("utf-8") for c in charset]
    n, width = len(syms), max(len(s) for s in syms)
    table = np.zeros((n, width), dtype=np.uint8)
    for k, s in enumerate(syms):
        table[k, :len(s)] = np.frombuffer(s, dtype=np.uint8)
    slen = np.array([len(s) for s in syms], dtype=np.int64)
    idx = np.arange(count, dtype=np.uint64) + np.uint64(start)
    digits = np.empty((length, count), dtype=np.int64)          # [position][candidate], most significant first
    for p in range(length - 1, -1, -1):
        digits[p] = (idx % np.uint64(n)).astype(np.int64)
        idx //= np.uint64(n)
    lens = slen[digits]
    offs = np.zeros(count + 1, dtype=np.uint64)
    np.cumsum(lens.sum(axis=0), out=offs[1:])
    blob = np.empty(int(offs[-1]), dtype=np.uint8)
    cur = offs[:-1].astype(np.int64)
    for p in range(length):
        d, lp = digits[p], lens[p]
        if width == 1 or (lp == lp[0]).all():
            for b in range(int(lp[0]) if width > 1 else 1):
                blob[cur + b] = table[d, b]
        else:
            for b in range(width):
                m = lp > b
                blob[cur[m] + b] = table[d[m], b]
        cur += lp
    return blob.tobytes(), offs


def spell_utf8_parallel(charset, length, start, count, workers=8, part=1 << 18):
    """spell_utf8 over sub-windows on a thread pool (numpy releases the GIL in the gathers and scatters): ~3x the
    single-thread rate on 8 cores, so a multi-byte charset's host spelling keeps up with the slower formats."""
    if count <= part or workers <= 1:
        return spell_utf8(charset, length, start, count)
    from concurrent.futures import ThreadPoolExecutor
    bounds = [(s, min(part, start + count - s)) for s in range(start, start + count, part)]
    with ThreadPoolExecutor(max_workers=workers) as ex:
        res = list(ex.map(lambda b: spell_utf8(charset, length, b[0], b[1]), bounds))
    offs = [res[0][1]]
    base = res[0][1][-1]
    for _, o in res[1:]:
        offs.append(o[1:] + base)
        base += o[-1]
    return b"".join(b for b, _ in res), np.concatenate(offs)


def build_message(stream, charset, segments):
    """The server's JSON payload for these segments, as bytes (same text json.dumps gives, key order
    data, passwords)."""
    if not _json_safe(charset):
        pw = []
        ks = Keyspace(charset, max(L for L, _, _ in segments))
        for L, s, c in segments:
            pw.extend(ks.password(L, s + k) for k in range(c))
        return json.dumps({"data": stream, "passwords": pw}).encode()
    parts = []
    for L, s, c in segments:
        if c <= 0:
            continue
        row = np.empty((c, L + 4), dtype=np.uint8)
        row[:, 0] = 0x22
        segment_chars(charset, L, s, c, out=row[:, 1:L + 1])
        row[:, L + 1] = 0x22
        row[:, L + 2] = 0x2C
        row[:, L + 3] = 0x20
        parts.append(row.tobytes())
    body = b"".join(parts)[:-2] if parts else b""
    return b'{"data": ' + json.dumps(stream).encode() + b', "passwords": [' + body + b"]}"


def _pack(strings):
    bs = [s.encode("utf-8") for s in strings]
    offs = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        np.cumsum([len(b) for b in bs], out=offs[1:])
    return b"".join(bs), offs


def parse_message(raw):
    """(stream, blob, offsets) of a server payload; candidate k is blob[offsets[k]:offsets[k+1]]
    (UTF-8).  Without escapes in the text, every '"' delimits a string: the strings are cut out with
    numpy.  Anything else goes through json.loads."""
    if isinstance(raw, str):
        raw = raw.encode("utf-8")
    if b"\\" not in raw:
        a = np.frombuffer(raw, dtype=np.uint8)
        q = np.flatnonzero(a == 0x22)
        if len(q) >= 6 and len(q) % 2 == 0:
            opens, closes = q[0::2], q[1::2]
            # keys are the strings followed by ':'
            nxt = np.minimum(closes + 1, len(a) - 1)
            keymask = a[nxt] == 0x3A
            keys = np.flatnonzero(keymask)
            if len(keys) == 2:
                names = [raw[opens[k] + 1:closes[k]] for k in keys]
                if sorted(names) == [b"data", b"passwords"]:
                    kd = keys[names.index(b"data")]
                    kp = keys[names.index(b"passwords")]
                    stream = raw[opens[kd + 1] + 1:closes[kd + 1]].decode("utf-8")
                    if kp > kd:
                        lo, hi = kp + 1, len(opens)
                    else:
                        lo, hi = kp + 1, kd
                    st = opens[lo:hi] + 1
                    ln = closes[lo:hi] - st
                    offs = np.zeros(len(st) + 1, dtype=np.uint64)
                    np.cumsum(ln, out=offs[1:])
                    return stream, _cut(a, st, ln, offs), offs
    d = json.loads(raw)
    blob, offs = _pack(d["passwords"])
    return d["data"], blob, offs


def _cut(a, st, ln, offs):
    """Concatenate a[st[k]:st[k]+ln[k]] for all k.  Runs of equally long strings at a constant stride
    (what a server segment produces) are cut with one strided view each; the rest with a gather."""
    n = len(st)
    if n == 0 or int(offs[-1]) == 0:
        return b""
    # break points: where the length or the stride changes
    stride = np.diff(st)
    brk = np.flatnonzero((ln[1:] != ln[:-1]) | (np.diff(stride, prepend=stride[:1]) != 0)) + 1 if n > 1 else []
    bounds = [0] + [int(b) for b in brk] + [n]
    parts = []
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        L = int(ln[b0])
        if b1 - b0 >= 2 and L > 0:
            S = int(st[b0 + 1] - st[b0])
            if S >= L and int(st[b1 - 1]) == int(st[b0]) + S * (b1 - b0 - 1):
                v = np.lib.stride_tricks.as_strided(a[int(st[b0]):], shape=(b1 - b0, L), strides=(S, 1))
                parts.append(np.ascontiguousarray(v).tobytes())
                continue
        for k in range(b0, b1):
            parts.append(a[int(st[k]):int(st[k]) + int(ln[k])].tobytes())
    return b"".join(parts)


def candidate(blob, offsets, k):
    return bytes(blob[int(offsets[k]):int(offsets[k + 1])]).decode("utf-8")

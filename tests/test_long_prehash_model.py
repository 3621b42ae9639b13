"""CPU restatement of k_long_prehash's message construction (dprf_amd/csrc/dprf_kernels.hip, DPRF_PART_LONG) against
hashlib: a record of any length, read as 16-byte aligned LE words of a blob, with an optional 16-byte BE prefix (Office
H0 = SHA1(salt || UTF-16LE)) or an 8-byte suffix (PDF R5 / R6: SHA256(pw || salt8)), the 0x80 terminator and the bit
length -- every message word built the way the kernel builds it (word index t of block b, the suffix words shifted in
at byte offset len).  Lengths 0..300 cover every block-boundary case (55/56/63/64 ... past the prefix / suffix)."""
import hashlib
import random
import struct

M32 = 0xffffffff


def le_keep_mask(n):
    return 0 if n <= 0 else (M32 if n >= 4 else (1 << (8 * n)) - 1)


def long_msg_word(rec, length, dw, sw, ns):
    v = rec[dw] & le_keep_mask(length - 4 * dw) if 4 * dw < length else 0
    q, r = length >> 2, (length & 3) * 8
    for k in range(3):
        if k >= ns:
            break
        if dw == q + k:
            v |= (sw[k] << r) & M32
        if r and dw == q + k + 1:
            v |= sw[k] >> (32 - r)
    return v


def bswap(x):
    return struct.unpack("<I", struct.pack(">I", x))[0]


def sha1_compress(h, w):
    w = list(w)
    for t in range(16, 80):
        x = w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16]
        w.append(((x << 1) | (x >> 31)) & M32)
    a, b, c, d, e = h
    for t in range(80):
        if t < 20:
            f, k = (b & c) | (~b & d), 0x5A827999
        elif t < 40:
            f, k = b ^ c ^ d, 0x6ED9EBA1
        elif t < 60:
            f, k = (b & c) | (b & d) | (c & d), 0x8F1BBCDC
        else:
            f, k = b ^ c ^ d, 0xCA62C1D6
        tmp = (((a << 5) | (a >> 27)) + (f & M32) + e + k + w[t]) & M32
        e, d, c, b, a = d, c, ((b << 30) | (b >> 2)) & M32, a, tmp
    return [(x + y) & M32 for x, y in zip(h, (a, b, c, d, e))]


K256 = [int(x, 16) for x in (
    "428a2f98 71374491 b5c0fbcf e9b5dba5 3956c25b 59f111f1 923f82a4 ab1c5ed5 d807aa98 12835b01 243185be 550c7dc3 "
    "72be5d74 80deb1fe 9bdc06a7 c19bf174 e49b69c1 efbe4786 0fc19dc6 240ca1cc 2de92c6f 4a7484aa 5cb0a9dc 76f988da "
    "983e5152 a831c66d b00327c8 bf597fc7 c6e00bf3 d5a79147 06ca6351 14292967 27b70a85 2e1b2138 4d2c6dfc 53380d13 "
    "650a7354 766a0abb 81c2c92e 92722c85 a2bfe8a1 a81a664b c24b8b70 c76c51a3 d192e819 d6990624 f40e3585 106aa070 "
    "19a4c116 1e376c08 2748774c 34b0bcb5 391c0cb3 4ed8aa4a 5b9cca4f 682e6ff3 748f82ee 78a5636f 84c87814 8cc70208 "
    "90befffa a4506ceb bef9a3f7 c67178f2").split()]


def ror(x, n):
    return ((x >> n) | (x << (32 - n))) & M32


def sha256_compress(h, w):
    w = list(w)
    for t in range(16, 64):
        s0 = ror(w[t - 15], 7) ^ ror(w[t - 15], 18) ^ (w[t - 15] >> 3)
        s1 = ror(w[t - 2], 17) ^ ror(w[t - 2], 19) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & M32)
    a, b, c, d, e, f, g, hh = h
    for t in range(64):
        t1 = (hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K256[t] + w[t]) & M32
        t2 = ((ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M32
        hh, g, f, e, d, c, b, a = g, f, e, (d + t1) & M32, c, b, a, (t1 + t2) & M32
    return [(x + y) & M32 for x, y in zip(h, (a, b, c, d, e, f, g, hh))]


def kernel_prehash(data, prefix=None, suffix=None):
    """The kernel's loop for one lane: record words from a 16-byte aligned, zero-padded record."""
    padded = data + bytes((-len(data)) % 16)
    rec = list(struct.unpack("<%dI" % (len(padded) // 4), padded)) or [0]
    sha1 = prefix is not None
    prew = 4 if sha1 else 0
    salt = suffix is not None
    sw = [struct.unpack("<I", suffix[:4])[0], struct.unpack("<I", suffix[4:])[0], 0x80] if salt else [0x80, 0, 0x80]
    ns = 3 if salt else 1
    total = 4 * prew + len(data) + (8 if salt else 0)
    nb = (total + 9 + 63) >> 6
    h = [0x67452301, 0xEFCDAB89, 0x98BADCFE, 0x10325476, 0xC3D2E1F0] if sha1 else \
        [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
    pre = list(struct.unpack(">4I", prefix)) if sha1 else None
    for b in range(nb):
        w = []
        for j in range(16):
            t = 16 * b + j
            w.append(pre[j & 3] if t < prew else bswap(long_msg_word(rec, len(data), t - prew, sw, ns)))
        if b + 1 == nb:
            w[14], w[15] = 0, (total * 8) & M32
        h = sha1_compress(h, w) if sha1 else sha256_compress(h, w)
    return b"".join(struct.pack(">I", x) for x in h)


def test_long_prehash_model_matches_hashlib():
    rng = random.Random(4)
    salt16, salt8 = bytes(rng.getrandbits(8) for _ in range(16)), bytes(rng.getrandbits(8) for _ in range(8))
    for n in list(range(0, 140)) + [175, 176, 177, 199, 200, 255, 256, 300, 1000]:
        data = bytes(rng.getrandbits(8) or 1 for _ in range(n))
        assert kernel_prehash(data) == hashlib.sha256(data).digest(), ("sha256", n)
        assert kernel_prehash(data, suffix=salt8) == hashlib.sha256(data + salt8).digest(), ("sha256+salt", n)
        if n % 2 == 0:                                   # Office records are UTF-16LE: even lengths
            assert kernel_prehash(data, prefix=salt16) == hashlib.sha1(salt16 + data).digest(), ("sha1", n)

"""CPU restatement of the PDF R6 kernel's lane-group split AES (dprf_amd/csrc/dprf_kernels_r6.hip,
aes128_expand_split / aes128_encrypt_split / r6_round_asm), checked against FIPS-197 and a plain T-table AES.

The kernel replicates four T-tables T_t = ror(Te0, 8t) 16 times per 256-byte row and lets lane group A (bit 4 of
the lane clear) read T_t and group B read T_t+1 in every lookup, so a 32-lane ds_read_b32 half meets 32 banks.
B keeps its state rotated -- after round r its register j holds ror(s_(j + rho_r), 8 eps_r) -- and one uniform
instruction stream stays correct for both groups.  This test runs exactly that instruction stream for both groups
(same register, same byte, per-group table and round-key permutation, the final v_perm un-rotation) and pins the
constants the kernel uses (the (rho, eps) table and the lane base words) by reading them from the source.
"""
import os
import random
import re

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "dprf_amd", "csrc", "dprf_kernels_r6.hip")
M = 0xffffffff


def _sbox():
    sb = [0] * 256
    p = q = 1
    sb[0] = 0x63
    while True:
        p = (p ^ ((p << 1) & 0xff) ^ (0x1b if p & 0x80 else 0)) & 0xff
        q ^= q << 1
        q ^= q << 2
        q ^= q << 4
        q &= 0xff
        if q & 0x80:
            q ^= 0x09
        x = q ^ ((q << 1 | q >> 7) & 0xff) ^ ((q << 2 | q >> 6) & 0xff) ^ ((q << 3 | q >> 5) & 0xff) ^ \
            ((q << 4 | q >> 4) & 0xff)
        sb[p] = (x ^ 0x63) & 0xff
        if p == 1:
            return sb


SB = _sbox()


def xt(a):
    return ((a << 1) ^ (0x1b if a & 0x80 else 0)) & 0xff


def ror(x, n):
    n %= 32
    return ((x >> n) | (x << (32 - n))) & M


def rol(x, n):
    return ror(x, 32 - n % 32)


def byte(x, k):
    return (x >> (8 * k)) & 0xff


TE0 = [(xt(SB[x]) << 24) | (SB[x] << 16) | (SB[x] << 8) | (xt(SB[x]) ^ SB[x]) for x in range(256)]
T = [[ror(TE0[x], 8 * t) for x in range(256)] for t in range(4)]


def expand(key):
    rk = list(key)
    rcon = [1, 2, 4, 8, 16, 32, 64, 128, 0x1b, 0x36]
    for i in range(10):
        t = rol(rk[4 * i + 3], 8)
        sw = (SB[byte(t, 3)] << 24) | (SB[byte(t, 2)] << 16) | (SB[byte(t, 1)] << 8) | SB[byte(t, 0)]
        rk.append(rk[4 * i] ^ sw ^ (rcon[i] << 24))
        for k in range(3):
            rk.append(rk[-1] ^ rk[4 * i + 1 + k])
    return rk


def encrypt_plain(rk, pt):
    s = [pt[k] ^ rk[k] for k in range(4)]
    for r in range(1, 10):
        s = [T[0][byte(s[j], 3)] ^ T[1][byte(s[(j + 1) % 4], 2)] ^ T[2][byte(s[(j + 2) % 4], 1)] ^
             T[3][byte(s[(j + 3) % 4], 0)] ^ rk[4 * r + j] for j in range(4)]
    return [((SB[byte(s[j], 3)] << 24) | (SB[byte(s[(j + 1) % 4], 2)] << 16) | (SB[byte(s[(j + 2) % 4], 1)] << 8) |
             SB[byte(s[(j + 3) % 4], 0)]) ^ rk[40 + j] for j in range(4)]


def kernel_tables():
    src = open(SRC).read()
    rho = [int(v) for v in re.search(r"R6_RHO\[11\] = \{([^}]*)\}", src).group(1).split(",")]
    eps = [int(v) for v in re.search(r"R6_EPS\[11\] = \{([^}]*)\}", src).group(1).split(",")]
    m = re.search(r"S\.base = c4 \+ \(gb \? (0x[0-9a-f]+)u : (0x[0-9a-f]+)u\)", src)
    return rho, eps, int(m.group(2), 16), int(m.group(1), 16)      # base words of group A, group B


def perm(src0, src1, sel):
    """v_perm_b32: selector byte 0-3 -> src1 bytes, 4-7 -> src0 bytes, 0x0c -> 0"""
    out = 0
    for k in range(4):
        s = byte(sel, k)
        v = byte(src1, s) if s < 4 else (byte(src0, s - 4) if s < 8 else 0)
        out |= v << (8 * k)
    return out


def encrypt_split(rk, pt, group, lanec):
    """The kernel's instruction stream for one lane: lanec = 4 * (lane % 16), group 0 = A, 1 = B."""
    rho, eps, base_a, base_b = kernel_tables()
    base = (lanec * 0x01010101 + (base_b if group else base_a)) & M
    # tables are addressed by row x (byte 1) and byte 0 = 4 * (16 t + c): decode which table a lookup reads
    def lookup(v, K, I):
        a = perm(v, base, 0x0c0c0000 | ((4 + K) << 8) | I)
        x, col = a >> 8, (a & 0xff) // 4
        assert col % 16 == lanec // 4
        return T[col // 16][x], col // 16
    rkb = list(rk)
    sk = [0x03020100, 0x00030201, 0x01000302, 0x02010003]
    for r in range(1, 11):
        kk = rk[4 * r:4 * r + 4]
        for j in range(4):
            rkb[4 * r + j] = perm(kk[j], kk[(j + rho[r]) % 4], sk[eps[r]] if group else 0x07060504)
    s = [pt[k] ^ rkb[k] for k in range(4)]
    tables_used = set()
    for r in range(1, 10):
        n = []
        for j in range(4):
            acc = rkb[4 * r + j]
            for t in range(4):
                v, tab = lookup(s[(j + t) % 4], 3 - t, t)
                tables_used.add((t, tab))
                acc ^= v
            n.append(acc)
        s = n
    acc = []
    for j in range(4):
        x3, _ = lookup(s[j], 3, 2)
        x2, _ = lookup(s[(j + 1) % 4], 2, 3)
        x1, _ = lookup(s[(j + 2) % 4], 1, 0)
        x0, _ = lookup(s[(j + 3) % 4], 0, 1)
        acc.append((perm(x3, x2, 0x07020c0c) | perm(x1, x0, 0x0c0c0500)) ^ rkb[40 + j])
    selr = 0x02010003 if (base & 0x40) else 0x07060504
    return [perm(acc[j], acc[(j + 3) % 4], selr) for j in range(4)], tables_used


def test_fips197_vector_both_groups():
    rk = expand([0x00010203, 0x04050607, 0x08090a0b, 0x0c0d0e0f])
    pt = [0x00112233, 0x44556677, 0x8899aabb, 0xccddeeff]
    want = [0x69c4e0d8, 0x6a7b0430, 0xd8cdb780, 0x70b4c55a]
    assert encrypt_plain(rk, pt) == want
    for g in (0, 1):
        for c in (0, 4, 60):
            assert encrypt_split(rk, pt, g, c)[0] == want


def test_random_blocks_and_bank_disjointness():
    rng = random.Random(6)
    for _ in range(40):
        rk = expand([rng.getrandbits(32) for _ in range(4)])
        pt = [rng.getrandbits(32) for _ in range(4)]
        ref = encrypt_plain(rk, pt)
        a, ta = encrypt_split(rk, pt, 0, 4 * rng.randrange(16))
        b, tb = encrypt_split(rk, pt, 1, 4 * rng.randrange(16))
        assert a == ref and b == ref
        # lookup index t reads T_t in group A and T_t+1 in group B: their 16 copies sit in banks 16t..16t+15 and
        # 16(t+1).. (mod 32 for ds_read_b32), so the two halves of a 32-lane access never share a bank
        da, db = dict(ta), dict(tb)
        for t in range(4):
            assert da[t] == t and db[t] == (t + 1) % 4
            assert (16 * da[t]) % 32 != (16 * db[t]) % 32


def test_key_schedule_lookups_both_groups():
    """aes128_expand_split: byte p of SubWord(RotWord(t)) through base byte 1-p (A: T_1-p, B: T_2-p, both holding
    S[x] at byte p), combined by the same two v_perm as the last round."""
    _, _, base_a, base_b = kernel_tables()
    rng = random.Random(7)
    rcon = [1, 2, 4, 8, 16, 32, 64, 128, 0x1b, 0x36]
    for _ in range(20):
        key = [rng.getrandbits(32) for _ in range(4)]
        for g, lanec in ((0, 8), (1, 52)):
            base = (lanec * 0x01010101 + (base_b if g else base_a)) & M

            def lk(v, K, I):
                a = perm(v, base, 0x0c0c0000 | ((4 + K) << 8) | I)
                return T[(a & 0xff) // 64][a >> 8]
            rk = list(key)
            for i in range(10):
                t = rk[4 * i + 3]
                sw = perm(lk(t, 2, 2), lk(t, 1, 3), 0x07020c0c) | perm(lk(t, 0, 0), lk(t, 3, 1), 0x0c0c0500)
                rk.append(rk[4 * i] ^ sw ^ (rcon[i] << 24))
                for k in range(3):
                    rk.append(rk[-1] ^ rk[4 * i + 1 + k])
            assert rk == expand(key)

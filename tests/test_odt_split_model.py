"""CPU restatement of the ODF check kernel's split-table AES-256 decryption (dprf_amd/csrc/dprf_kernels.hip,
ODT_SPLIT: odt_round_asm / odt_dk_split / aes256_decrypt_split), checked against FIPS-197 C.3 and a plain
T-table inverse cipher for both lane groups.  Group A reads Td_t, group B Td_t+1 in every lookup; B carries its
state rotated (register j = ror(s_(j + rho_r), 8 eps_r), (rho, eps) -> (rho - eps, eps + 1) per inner round of the
inverse cipher), its round keys are permuted to match and one v_perm per word undoes the rotation at the end.  The
(rho, eps) table and the lane base words are read from the kernel source."""
import os
import random
import re

from test_r6_split_model import SB, byte, perm, rol, ror, xt

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "..", "dprf_amd", "csrc", "dprf_kernels.hip")
SI = [0] * 256
for _x in range(256):
    SI[SB[_x]] = _x


def mul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a = xt(a)
        b >>= 1
    return r


TD0 = [(mul(SI[x], 14) << 24) | (mul(SI[x], 9) << 16) | (mul(SI[x], 13) << 8) | mul(SI[x], 11) for x in range(256)]
TD = [[ror(TD0[x], 8 * t) for x in range(256)] for t in range(4)]


def expand256(key):
    rk, rcon, i = list(key), [1, 2, 4, 8, 16, 32, 64], 8
    while len(rk) < 60:
        t = rk[-1]
        if i % 8 == 0:
            t = rol(t, 8)
            t = (SB[byte(t, 3)] << 24) | (SB[byte(t, 2)] << 16) | (SB[byte(t, 1)] << 8) | SB[byte(t, 0)]
            t ^= rcon[i // 8 - 1] << 24
        elif i % 8 == 4:
            t = (SB[byte(t, 3)] << 24) | (SB[byte(t, 2)] << 16) | (SB[byte(t, 1)] << 8) | SB[byte(t, 0)]
        rk.append(rk[-8] ^ t)
        i += 1
    return rk


def dec_schedule(rk):
    def invmix(w):
        return TD[0][SB[byte(w, 3)]] ^ TD[1][SB[byte(w, 2)]] ^ TD[2][SB[byte(w, 1)]] ^ TD[3][SB[byte(w, 0)]]
    dk = []
    for r in range(14, -1, -1):
        ws = rk[4 * r:4 * r + 4]
        dk += [invmix(w) for w in ws] if 0 < r < 14 else ws
    return dk


def decrypt_plain(dk, ct):
    s = [ct[k] ^ dk[k] for k in range(4)]
    for r in range(1, 14):
        s = [TD[0][byte(s[j], 3)] ^ TD[1][byte(s[(j - 1) % 4], 2)] ^ TD[2][byte(s[(j - 2) % 4], 1)] ^
             TD[3][byte(s[(j - 3) % 4], 0)] ^ dk[4 * r + j] for j in range(4)]
    return [((SI[byte(s[j], 3)] << 24) | (SI[byte(s[(j - 1) % 4], 2)] << 16) | (SI[byte(s[(j - 2) % 4], 1)] << 8) |
             SI[byte(s[(j - 3) % 4], 0)]) ^ dk[56 + j] for j in range(4)]


def kernel_constants():
    src = open(SRC).read()
    rho = [int(v) for v in re.search(r"ODT_RHO\[14\] = \{([^}]*)\}", src).group(1).split(",")]
    eps = [int(v) for v in re.search(r"ODT_EPS\[14\] = \{([^}]*)\}", src).group(1).split(",")]
    m = re.search(r"base = lanec \* 0x01010101u \+ \(\(threadIdx\.x & 16u\) \? (0x[0-9a-f]+)u : (0x[0-9a-f]+)u\)", src)
    return rho, eps, int(m.group(2), 16), int(m.group(1), 16)


def decrypt_split(dk, ct, group, lanec):
    """The kernel's instruction stream for one lane (lanec = 4 * (lane % 16))."""
    rho, eps, base_a, base_b = kernel_constants()
    base = (lanec * 0x01010101 + (base_b if group else base_a)) & 0xffffffff
    sk = [0x03020100, 0x00030201, 0x01000302, 0x02010003]
    dkb = list(dk)
    gb = bool(base & 0x40)
    for r in range(1, 15):
        rr, ee = (rho[r], eps[r]) if r < 14 else (rho[13] - eps[13], eps[13])
        kk = dk[4 * r:4 * r + 4]
        for j in range(4):
            dkb[4 * r + j] = perm(kk[j], kk[(j + rr) % 4], sk[ee] if gb else 0x07060504)

    def lookup(v, t):
        a = perm(v, base, 0x0c0c0000 | ((4 + 3 - t) << 8) | t)
        col = (a & 0xff) // 4
        assert col % 16 == lanec // 4
        return TD[col // 16][a >> 8], col // 16
    s = [ct[k] ^ dkb[k] for k in range(4)]
    used = set()
    for r in range(1, 14):
        n = []
        for j in range(4):
            acc = dkb[4 * r + j]
            for t in range(4):
                v, tab = lookup(s[(j - t) % 4], t)
                used.add((t, tab))
                acc ^= v
            n.append(acc)
        s = n
    acc = [((SI[byte(s[j], 3)] << 24) | (SI[byte(s[(j + 3) % 4], 2)] << 16) | (SI[byte(s[(j + 2) % 4], 1)] << 8) |
            SI[byte(s[(j + 1) % 4], 0)]) ^ dkb[56 + j] for j in range(4)]
    selr = 0x02010003 if gb else 0x07060504
    return [perm(acc[j], acc[(j + 3) % 4], selr) for j in range(4)], used


def test_fips197_c3_both_groups():
    key = [0x00010203, 0x04050607, 0x08090a0b, 0x0c0d0e0f, 0x10111213, 0x14151617, 0x18191a1b, 0x1c1d1e1f]
    ct = [0x8ea2b7ca, 0x516745bf, 0xeafc4990, 0x4b496089]
    dk = dec_schedule(expand256(key))
    want = [0x00112233, 0x44556677, 0x8899aabb, 0xccddeeff]
    assert decrypt_plain(dk, ct) == want
    for g in (0, 1):
        for c in (0, 28, 60):
            assert decrypt_split(dk, ct, g, c)[0] == want


def test_random_blocks_and_tables():
    rng = random.Random(14)
    for _ in range(30):
        dk = dec_schedule(expand256([rng.getrandbits(32) for _ in range(8)]))
        ct = [rng.getrandbits(32) for _ in range(4)]
        ref = decrypt_plain(dk, ct)
        a, ua = decrypt_split(dk, ct, 0, 4 * rng.randrange(16))
        b, ub = decrypt_split(dk, ct, 1, 4 * rng.randrange(16))
        assert a == ref and b == ref
        assert dict(ua) == {t: t for t in range(4)} and dict(ub) == {t: (t + 1) % 4 for t in range(4)}

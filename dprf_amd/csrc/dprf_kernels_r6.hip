/* dprf_kernels_r6.hip -- PDF 1.7 ext-3 / 2.0 revision 6 hardened hash, one candidate per lane.
 *
 * Restates pdf_compute_hardened_hash_r6 (pdf_password_verifier.c:226-291, ownerkey == NULL) and the
 * U[0:32] compare (:115-132):
 *     K = SHA256(pw || U[32:40]); bs = 32
 *     round i = 0, 1, ...:  data = 64 x (pw || K[0:bs])
 *                           E = AES-128-CBC-encrypt(key K[0:16], iv K[16:32], data)
 *                           bs = 32 + 16 * (sum(E[0:16]) mod 3)
 *                           K = SHA-256 / SHA-384 / SHA-512 (E)  (by bs)
 *                           stop once i+1 >= 64 and i+1 >= E[last] + 32           (:247)
 *
 * Design:
 *  - `data` is never materialised.  Each lane keeps one period P = pw || K[0:bs] plus P[0:16] again in
 *    its own LDS bank column ([word][lane], so a lane's words share one bank) and pulls each 16-byte
 *    block out of it with 5 ds_read_b32 + 4 v_perm; ciphertext goes straight into the SHA message
 *    registers 64 bytes (4 AES blocks) at a time.
 *  - AES T-tables: four rotated copies of Te0, 16 copies each, read by two lane groups from different tables so
 *    every lookup is conflict-free and no rotates remain (aes128_encrypt_split); inner rounds as asm blocks.
 *  - Slots and classes: a workgroup holds more candidates ("slots") than lanes, every slot's period and state in
 *    LDS; a round runs for 64 queued slots of one hash class, so the SHA-256 / SHA-384 / SHA-512 choice and the
 *    round's length never diverge inside a wave (the flow scheduler below, r6_claim).
 *  - Persistent workgroups: a slot whose candidate finishes takes the next one from the launch's cursor.
 */
#include "dev_crypto.h"
#include "dprf_params.h"
#include "dprf_launch.h"
#include "dprf_hits.h"

#include <mutex>

/* T-tables in 256-byte rows, row x = entry x: four tables T_t = ror(Te0, 8t), 16 copies each, copy c of T_t at byte
 * 256 x + 4 (16 t + c); the address of a lookup is ONE v_perm (below).  Lane groups A (bit 4 of the lane clear) and B
 * read different tables in every lookup, so the 32 lanes of a ds_read_b32 half ({0-31}, {32-63}: MI355X_MICROARCH.md
 * LDS table) meet 32 different banks, and no rotates are left (aes128_encrypt_split).  Measured against the layouts of
 * rounds 1-2 (one table x 32 copies 3.02 M cand/s, Te0 + Te2 x 32 copies 3.50 M, four tables x 8 copies 1.91 M: bank
 * conflicts cost more than rotates; HISTORY.md) -- the split layout took R6 to 3.68 M in round 3. */
#define R6_TE_ROW_BYTES 256
#define R6_TABLES 4
#define R6_TE_COPIES 16
#define R6_TE_BYTES (256 * R6_TE_ROW_BYTES)
/* bytes of a row the tables take (the whole row: no slot periods beside them, slot_lds te_slots = 0) */
#define R6_TE_USED (4 * R6_TABLES * R6_TE_COPIES)
static_assert(R6_TE_USED <= R6_TE_ROW_BYTES && (R6_TE_COPIES & (R6_TE_COPIES - 1)) == 0, "table rows");

DEVI uint32_t fastdiv6(uint32_t n, uint32_t m, uint32_t s) {
    uint32_t t = __umulhi(n, m);
    return (t + ((n - t) >> 1)) >> s;
}

/* static, so its LDS address is a link-time constant (0) and folds into the ds_read: the v_perm result is
 * the whole address */
__shared__ __attribute__((aligned(16))) uint32_t r6_te[R6_TE_BYTES / 4];

/* LDS pointers from 32-bit LDS byte addresses (address space 3: ds_* instructions, no flat pointers) */
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) uint32_t lds_u32;
DEVI lds_u8 *L8(uint32_t a) { return (lds_u8 *)(size_t)a; }
DEVI lds_u32 *L32(uint32_t a) { return (lds_u32 *)(size_t)a; }
DEVI uint32_t lds_addr(const void *p) { return (uint32_t)(size_t)(const lds_u8 *)p; }

/* the lane index as an opaque value (LLVM cannot hoist it): used where a lane-derived value would otherwise be held
 * across the persistent loop -- at the kernel's VGPR limit such values were what the register allocator spilled */
DEVI uint32_t opaque_lane() {
    uint32_t l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

struct r6_lds {
    uint32_t pat;              /* LDS byte address of the slot's group: rows of 256 bytes */
    uint32_t lanebase;         /* 4 * (slot % 64): the slot's column in the pattern area */
    uint32_t lanec;            /* 4 * (thread lane % R6_TE_COPIES): this thread's table copy */
    uint32_t base;             /* byte t: row offset of the copy of the table lookup t reads (A: T_t, B: T_t+1) */
};

DEVI uint32_t pat_addr(uint32_t pos, uint32_t lanebase) { return ((pos >> 2) << 8) | (pos & 3u) | lanebase; }

/* Lane-group split AES (round 3).  Four tables T_t = ror(Te0, 8t), 16 copies each: copy c of T_t is dword 16t + c
 * of every 256-byte row, so it sits in bank (16t + c) mod 32 of a ds_read_b32 (MI355X_MICROARCH.md LDS table).
 * Lanes l (c = l % 16) form group A (bit 4 of l clear) and group B (set): in every lookup A reads T_t and B T_t+1,
 * so the 16 A lanes and the 16 B lanes of a 32-lane half meet 32 different banks.  B pays for reading the "wrong"
 * table by holding its state rotated: after round r its register j holds ror(s_(j + rho_r), 8 eps_r) (rho, eps
 * below), which one uniform instruction stream keeps consistent -- the byte K of register a that a lookup takes is,
 * for B, real byte K + eps of s_(a + rho), and T_t+1 supplies the real term rotated by the same amount for all four
 * terms of a column.  B's round keys are permuted to its representation once per key schedule, and the output
 * words are brought back by one v_perm each.  Against the two-table layout (Te0, Te2 x 32 copies) this removes the
 * four rotates of every round (72 issue slots per block) for four v_perm (8).  Checked on the CPU against FIPS-197
 * (tests/test_r6_split_model.py restates it). */
/* lookup: byte 1 of the address <- byte K of v, byte 0 <- byte I of the lane's base word (copy + table offset) */
template <int K, int I>
DEVI uint32_t r6_ld(uint32_t v, uint32_t base) {
    const uint32_t a = __builtin_amdgcn_perm(v, base, 0x0c0c0000u | ((4u + K) << 8) | I);
    return *(const uint32_t *)((const uint8_t *)r6_te + a);
}
/* B's representation (rho, eps) after round r = 0..10 */
__device__ constexpr int R6_RHO[11] = {0, 0, 1, 3, 2, 2, 3, 1, 0, 0, 1};
__device__ constexpr int R6_EPS[11] = {0, 1, 2, 3, 0, 1, 2, 3, 0, 1, 1};

DEVI void aes128_expand_split(const r6_lds &S, const uint32_t key[4], uint32_t rk[44]) {
    const uint32_t rcon[10] = {0x01000000u, 0x02000000u, 0x04000000u, 0x08000000u, 0x10000000u,
                               0x20000000u, 0x40000000u, 0x80000000u, 0x1b000000u, 0x36000000u};
    rk[0] = key[0]; rk[1] = key[1]; rk[2] = key[2]; rk[3] = key[3];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t t = rk[4 * i + 3];
        /* byte p of SubWord(RotWord(t)) = S[byte p-1 of t], from a table holding S at byte p: base byte 1-p names
         * T_1-p for A (S at bytes p+1, p) and T_2-p for B (S at bytes p, p-1) */
        const uint32_t sw = perm(r6_ld<2, 2>(t, S.base), r6_ld<1, 3>(t, S.base), 0x07020c0cu) |
                            perm(r6_ld<0, 0>(t, S.base), r6_ld<3, 1>(t, S.base), 0x0c0c0500u);
        rk[4 * i + 4] = rk[4 * i] ^ sw ^ rcon[i];
        rk[4 * i + 5] = rk[4 * i + 1] ^ rk[4 * i + 4];
        rk[4 * i + 6] = rk[4 * i + 2] ^ rk[4 * i + 5];
        rk[4 * i + 7] = rk[4 * i + 3] ^ rk[4 * i + 6];
    }
    /* group B: round r's key word j = ror(rk[4r + (j + rho_r) % 4], 8 eps_r); one v_perm per word (A: identity) */
    const bool gb = (S.base & 0x40u) != 0u;             /* byte 0: T_0 (A) or T_1 (B) */
    const uint32_t sk[4] = {gb ? 0x03020100u : 0x07060504u, gb ? 0x00030201u : 0x07060504u,
                            gb ? 0x01000302u : 0x07060504u, gb ? 0x02010003u : 0x07060504u};
#pragma unroll
    for (int r = 1; r <= 10; r++) {
        if (R6_RHO[r] == 0 && R6_EPS[r] == 0) continue;
        const uint32_t k0 = rk[4 * r], k1 = rk[4 * r + 1], k2 = rk[4 * r + 2], k3 = rk[4 * r + 3];
        const uint32_t kk[4] = {k0, k1, k2, k3};
#pragma unroll
        for (int j = 0; j < 4; j++) rk[4 * r + j] = perm(kk[j], kk[(j + R6_RHO[r]) & 3], sk[R6_EPS[r]]);
    }
}

/* One inner round as an asm block: the 16 lookups issued back to back (column by column), then each column's two
 * three-way XORs (v_bitop3 0x96) behind the wait that covers its four reads.  LLVM's schedule of the same dataflow keeps 1-2 reads in flight
 * per wait (the kernel sits at its VGPR limit) and exposes the LDS latency several times per round.  The block
 * ends with every read consumed, so no LDS operation of it is in flight for the compiler's own waits. */
#define R6_SEL(t) (0x0c0c0000u | ((4u + 3u - (t)) << 8) | (t))
/* The four lookups per round that take byte 1 of a state word (term t = 2) form their
 * address as (s & 0xff00) | (base >> 16 without its byte 1) -- ONE v_bitop3 (truth table 0xe2, full rate on gfx950
 * with two VGPR sources) instead of a v_perm (half rate); base >> 16 is formed once per round inside the block (a
 * long-lived register for it made the kernel spill 12 B/lane).  Measured: 3.743 -> 3.753 M cand/s (three alternating
 * runs, profiles/ab_r6_b1_bitop3_r04t.txt).  The other three terms need a shift first (v_lshrrev + v_bitop3 for bytes
 * 2 and 3, a half-rate v_lshlrev for byte 0): no fewer cycles than the v_perm. */
DEVI void r6_round_asm(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t base, uint32_t k0,
                       uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t t[16];
#define R6L(d, s, sel) "v_perm_b32 %" #d ", %" #s ", %20, %" #sel "\n\tds_read_b32 %" #d ", %" #d "\n\t"
    /* base >> 16 in t[15]'s register: its own lookup (the last of the 16) comes after the four that read it */
#define R6_B2PRE "v_lshrrev_b32 %19, 16, %20\n\t"
#define R6L2(d, s) "v_bitop3_b32 %" #d ", %" #s ", %29, %19 bitop3:0xe2\n\tds_read_b32 %" #d ", %" #d "\n\t"
#define R6_B2IN , "s"(0xff00u)
    asm volatile(
        /* column 0: s0 t0, s1 t1, s2 t2, s3 t3;  column 1: s1, s2, s3, s0;  column 2: s2, s3, s0, s1;  column 3 */
        R6_B2PRE
        R6L(4, 0, 25) R6L(5, 1, 26) R6L2(6, 2) R6L(7, 3, 28)
        R6L(8, 1, 25) R6L(9, 2, 26) R6L2(10, 3) R6L(11, 0, 28)
        R6L(12, 2, 25) R6L(13, 3, 26) R6L2(14, 0) R6L(15, 1, 28)
        R6L(16, 3, 25) R6L(17, 0, 26) R6L2(18, 1) R6L(19, 2, 28)
        "s_waitcnt lgkmcnt(12)\n\t"
        "v_bitop3_b32 %4, %4, %5, %6 bitop3:0x96\n\t"
        "v_bitop3_b32 %0, %4, %7, %21 bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(8)\n\t"
        "v_bitop3_b32 %8, %8, %9, %10 bitop3:0x96\n\t"
        "v_bitop3_b32 %1, %8, %11, %22 bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(4)\n\t"
        "v_bitop3_b32 %12, %12, %13, %14 bitop3:0x96\n\t"
        "v_bitop3_b32 %2, %12, %15, %23 bitop3:0x96\n\t"
        "s_waitcnt lgkmcnt(0)\n\t"
        "v_bitop3_b32 %16, %16, %17, %18 bitop3:0x96\n\t"
        "v_bitop3_b32 %3, %16, %19, %24 bitop3:0x96"
        : "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3), "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4]),
          "=&v"(t[5]), "=&v"(t[6]), "=&v"(t[7]), "=&v"(t[8]), "=&v"(t[9]), "=&v"(t[10]), "=&v"(t[11]),
          "=&v"(t[12]), "=&v"(t[13]), "=&v"(t[14]), "=&v"(t[15])
        : "v"(base), "v"(k0), "v"(k1), "v"(k2), "v"(k3), "s"(R6_SEL(0)), "s"(R6_SEL(1)), "s"(R6_SEL(2)),
          "s"(R6_SEL(3)) R6_B2IN
        : "memory");
#undef R6_B2IN
#undef R6_B2PRE
#undef R6L2
#undef R6L
}

/* E(v ^ iv): the CBC xor and the first AddRoundKey as one v_bitop3 per word (LLVM emits two v_xor) */
DEVI void aes128_encrypt_split(const r6_lds &S, const uint32_t rk[44], const uint32_t v[4], const uint32_t iv[4],
                               uint32_t out[4]) {
    uint32_t s[4] = {xor3(v[0], iv[0], rk[0]), xor3(v[1], iv[1], rk[1]), xor3(v[2], iv[2], rk[2]),
                     xor3(v[3], iv[3], rk[3])};
#pragma unroll
    for (int r = 1; r < 10; r++)
        r6_round_asm(s[0], s[1], s[2], s[3], S.base, rk[4 * r], rk[4 * r + 1], rk[4 * r + 2], rk[4 * r + 3]);
    /* last round: byte p of word j <- S[byte p of s_(j+3-p)] (B: of its rotated registers) through base byte 1-p
     * (A: T_1-p, B: T_2-p, both with S at byte p), combined as before (the compiler's schedule: an asm block like the
     * inner rounds' measured 3.666 vs 3.678 M cand/s, round 3) */
    uint32_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        acc[j] = (perm(r6_ld<3, 2>(s[j], S.base), r6_ld<2, 3>(s[(j + 1) & 3], S.base), 0x07020c0cu) |
                  perm(r6_ld<1, 0>(s[(j + 2) & 3], S.base), r6_ld<0, 1>(s[(j + 3) & 3], S.base), 0x0c0c0500u)) ^
                 rk[40 + j];
    /* B's word j holds ror(out[j + 1], 8): out[j] = rol(acc[j - 1], 8).  The selector is derived from base here
     * rather than kept in a register across the round (the kernel sits at its 168-VGPR limit) */
    const uint32_t selr = (S.base & 0x40u) ? 0x02010003u : 0x07060504u;
#pragma unroll
    for (int j = 0; j < 4; j++) out[j] = perm(acc[j], acc[(j + 3) & 3], selr);
}
#define R6_EXPAND aes128_expand_split
#define R6_ENCRYPT aes128_encrypt_split

/* SHA-512 over 32 BE words held as two 16-word halves; state as 16 BE words (hi, lo pairs) */
DEVI void sha512_compress_pairs(uint32_t hs[16], const uint32_t lo[16], const uint32_t hi[16]) {
    uint64_t st[8], w[16];
#pragma unroll
    for (int k = 0; k < 8; k++) st[k] = pack64(hs[2 * k], hs[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = pack64(lo[2 * k], lo[2 * k + 1]);
#pragma unroll
    for (int k = 0; k < 8; k++) w[8 + k] = pack64(hi[2 * k], hi[2 * k + 1]);
    sha512_compress(st, w);
#pragma unroll
    for (int k = 0; k < 8; k++) { hs[2 * k] = hi32(st[k]); hs[2 * k + 1] = lo32(st[k]); }
}

/* Load candidate `idx` (keyspace index or slot), compute K = SHA256(pw || salt), write pw to the
 * head of the lane's pattern column.  Returns the password length. */
/* MODE 2 (long list, round 4): the record (<= 176 bytes, pdf...c:228) is copied word by word into the period column
 * and K0 comes from k_long_prehash (keys, [8][ncand], launch-local candidate `off`). */
template <int MODE>
DEVI uint32_t r6_begin(const dprf_enum &e, const dprf_pdf_params &p, const uint8_t *cs, const uint8_t *sdig,
                       uint64_t idx, uint32_t off, const uint32_t *slots, const uint8_t *lens, const r6_lds &S,
                       uint32_t K[16], const uint64_t *loff = nullptr, const uint32_t *llen = nullptr,
                       const uint32_t *keys = nullptr, uint32_t ncand = 0) {
    if constexpr (MODE == 2) {
        const uint32_t len = llen[idx];
        const uint32_t *rec = slots + loff[idx];
        for (uint32_t k = 0; k < ((len + 3u) >> 2); k++) *L32(S.pat + ((k << 8) | S.lanebase)) = rec[k];
#pragma unroll
        for (int k = 0; k < 8; k++) K[k] = keys[(size_t)k * ncand + off];
#pragma unroll
        for (int k = 8; k < 16; k++) K[k] = 0u;
        return len;
    }
    uint32_t w[DPRF_SLOT_WORDS];
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) w[j] = 0;
    uint32_t len;
    if (MODE == 0) {
        /* a runtime loop over the pwlen positions (uniform), each character stored straight into the slot's
         * period column and the words read back: unrolled over DPRF_MAX_RANGE_LEN with the digits and the
         * words in registers, this once-per-candidate code spilled 300 B per lane in every wave of the
         * kernel (~2 KB of scratch writes per candidate, profiles/pmc_traffic.json r01) */
        uint32_t rem = off, carry = 0;
        const uint32_t n = e.pwlen;
#pragma unroll 1
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t pp = n - 1u - k;
            const uint32_t q = e.cslen == 1 ? rem : fastdiv6(rem, e.div_m, e.div_s);
            const uint32_t r = rem - q * e.cslen;
            uint32_t d = (uint32_t)sdig[pp] + r + carry;      /* LDS copy: a runtime index into the byval
                                                                 kernel argument would put it on the stack */
            carry = d >= e.cslen ? 1u : 0u;
            d -= carry ? e.cslen : 0u;
            rem = q;
            *L8(S.pat + pat_addr(pp, S.lanebase)) = cs[d];
        }
        len = n;
        /* opaque per-lane length: with the launch-uniform pwlen visible, LLVM hoists this once-per-candidate
         * SHA-256's uniform message words and K+W sums out of the persistent loop into ~70 long-lived VGPRs,
         * which then spill (~280 B per lane of scratch) */
        asm volatile("" : "+v"(len));
#pragma unroll
        for (int j = 0; j < DPRF_SLOT_WORDS; j++)
            w[j] = 4u * (uint32_t)j < len ? *L32(S.pat + (((uint32_t)j << 8) | S.lanebase)) : 0u;
    } else {
        const uint4 *s = (const uint4 *)(slots + idx * DPRF_SLOT_WORDS);
#pragma unroll
        for (int q = 0; q < DPRF_SLOT_WORDS / 4; q++) {
            uint4 v = s[q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        len = lens[idx];
    }
    /* K = SHA256(pw || salt8) (:240-245): LE message with the salt at byte offset len */
    uint32_t m[32];
#pragma unroll
    for (int j = 0; j < 32; j++) m[j] = j < DPRF_SLOT_WORDS ? (w[j] & le_keep_mask(j, len)) : 0u;
    const uint32_t sw[3] = {p.u[8], p.u[9], 0x80u};
    const uint32_t q = len >> 2, r = (len & 3u) * 8u;
#pragma unroll
    for (int s = 0; s < 3; s++) {
        const uint32_t lo = sw[s] << r;
        const uint32_t hi = r ? (sw[s] >> (32u - r)) : 0u;
#pragma unroll
        for (int j = 0; j < 32; j++) {
            if ((uint32_t)j == q + s) m[j] |= lo;
            if ((uint32_t)j == q + s + 1) m[j] |= hi;
        }
    }
    const uint32_t total = len + 8u, bits = total * 8u;
    const bool two = total > 55u;
    uint32_t b0[16], b1[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { b0[j] = bswap32(m[j]); b1[j] = bswap32(m[16 + j]); }
    if (!two) b0[15] = bits;
    b1[15] = bits;
    sha256_iv(K);
    sha256_compress(K, b0);
    if (two) sha256_compress(K, b1);
#pragma unroll
    for (int j = 8; j < 16; j++) K[j] = 0u;
    /* pw at the head of the period (word-aligned; bytes past len are overwritten by K) */
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) *L32(S.pat + (((uint32_t)j << 8) | S.lanebase)) = w[j];
    return len;
}

/* Write K[0:bs] (BE words) at byte `len` of the slot's period and repeat the period's first 16 bytes
 * after it (a 16-byte block read starting at o < Lp then never wraps). */
/* colbytes: the column's size in bytes -- the wrap copy stops there (range mode sizes the column to the bytes its
 * block reads can reach, launch_pdf_r6) */
DEVI void r6_store_k(const r6_lds &S, uint32_t len, uint32_t bs, const uint32_t K[16], uint32_t colbytes) {
#pragma unroll
    for (int k = 0; k < 64; k++) {
        if ((uint32_t)k < bs) {
            const uint32_t b = (K[k >> 2] >> (24 - 8 * (k & 3))) & 0xffu;
            *L8(S.pat + pat_addr(len + k, S.lanebase)) = (uint8_t)b;
        }
    }
    const uint32_t Lp = len + bs;
    for (uint32_t k = 0; k < 16 && Lp + k < colbytes; k++)
        *L8(S.pat + pat_addr(Lp + k, S.lanebase)) = *L8(S.pat + pat_addr(k, S.lanebase));
}

/* Four BE words starting at byte o of the slot's period (one v_perm per word). */
DEVI void r6_read16(const r6_lds &S, uint32_t o, uint32_t v[4]) {
    const uint32_t sel = 0x00010203u + (o & 3u) * 0x01010101u;
    const lds_u32 *col = L32(S.pat + (((o >> 2) << 8) | S.lanebase));
    uint32_t lw[5];
#pragma unroll
    for (int k = 0; k < 5; k++) lw[k] = col[k * 64];
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = perm(lw[k + 1], lw[k], sel);
}

/* K[0:32] of the slot (AES key and IV of the next round), read back from its period. */
DEVI void r6_load_k(const r6_lds &S, uint32_t len, uint32_t K[8]) {
    r6_read16(S, len, K);
    r6_read16(S, len + 16u, K + 4);
}

/* Hash family of the slot's next round: sum(E[0:16]) mod 3 of the first ciphertext block (:264-268). */
DEVI uint32_t r6_family(const r6_lds &S, uint32_t len) {
    uint32_t K[8], rk[44], v[4], y[4];
    r6_load_k(S, len, K);
    R6_EXPAND(S, K, rk);
    r6_read16(S, 0u, v);
    R6_ENCRYPT(S, rk, v, K + 4, y);
    uint32_t sum = __builtin_amdgcn_sad_u8(y[0], 0u, 0u);
    sum = __builtin_amdgcn_sad_u8(y[1], 0u, sum);
    sum = __builtin_amdgcn_sad_u8(y[2], 0u, sum);
    sum = __builtin_amdgcn_sad_u8(y[3], 0u, sum);
    return sum % 3u;
}

/* One round of the hardened hash for a slot whose family `hsel` is known: returns E[last]; K (16 BE
 * words, zero past the digest) and bs become the next round's; K[0:bs] is stored back into the period. */
/* UNI (range mode): every slot of a batch has the same period length (fixed pwlen, one bs per class) and
 * every batch one family, so Lp, the block offset o and the byte selector are wave-uniform scalars and a
 * block's LDS address is one v_add of the lane's column base (~15 VALU slots per AES block saved). */
template <bool UNI>
DEVI uint32_t r6_round(const r6_lds &S, uint32_t len, uint32_t &bs, uint32_t hsel, uint32_t K[16], uint32_t colbytes) {
    uint32_t Lp = len + bs;
    if (UNI) Lp = __builtin_amdgcn_readfirstlane(Lp);
    const uint32_t colbase = S.pat + S.lanebase;                 /* pat is only 16-byte aligned */
    r6_load_k(S, len, K);
    /* AES-128 key K[0:16], iv K[16:32] (:259-261) */
    uint32_t rk[44];
    R6_EXPAND(S, K, rk);
    uint32_t prev[4] = {K[4], K[5], K[6], K[7]};
    uint32_t hs[16], half[16];
    if (hsel == 0) {
        sha256_iv(hs);
    } else {
        uint64_t iv[8];
        sha512_iv(iv, hsel == 1);
#pragma unroll
        for (int k = 0; k < 8; k++) { hs[2 * k] = (uint32_t)(iv[k] >> 32); hs[2 * k + 1] = (uint32_t)iv[k]; }
    }
    uint32_t o = 0;
    for (uint32_t u = 0; u < Lp; u++) {         /* 64-byte units of data = 64 x period */
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint32_t v[4], y[4];
            if (UNI) {
                const uint32_t sel = 0x00010203u + (o & 3u) * 0x01010101u;
                const lds_u32 *col = L32(colbase + ((o >> 2) << 8));
                uint32_t lw[5];
#pragma unroll
                for (int k = 0; k < 4; k++) lw[k] = col[k * 64];
                /* the fifth word only for a block that does not start on a word (o is uniform: a scalar branch);
                 * the column ends where the aligned blocks' reads do (launch_pdf_r6) */
                lw[4] = (o & 3u) ? col[4 * 64] : lw[3];
#pragma unroll
                for (int k = 0; k < 4; k++) v[k] = perm(lw[k + 1], lw[k], sel);
            } else {
                r6_read16(S, o, v);
            }
            R6_ENCRYPT(S, rk, v, prev, y);
#pragma unroll
            for (int k = 0; k < 4; k++) { prev[k] = y[k]; w[4 * q + k] = y[k]; }
            o += 16u;
            o = o >= Lp ? o - Lp : o;
        }
        if (hsel == 0) {
            sha256_compress(hs, w);
        } else if (u & 1u) {
            sha512_compress_pairs(hs, half, w);
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) half[k] = w[k];
        }
    }
    const uint32_t bits = 64u * Lp * 8u;
    /* the padding word as an opaque value: LLVM otherwise folds the SHA-512 schedule terms of the constant padding
     * blocks into 64-bit constants held (and, at the VGPR limit, spilled) across the persistent loop */
    uint32_t pad = 0x80000000u;
    asm volatile("" : "+v"(pad));
    if (hsel == 0) {
        uint32_t w[16] = {pad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
        sha256_compress(hs, w);
#pragma unroll
        for (int k = 8; k < 16; k++) hs[k] = 0u;
    } else {
        uint32_t w[16] = {pad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
        if (Lp & 1u) {
            sha512_compress_pairs(hs, half, w);
        } else {
            uint32_t z[16] = {pad, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t w2[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
            sha512_compress_pairs(hs, z, w2);
        }
        if (hsel == 1) {
#pragma unroll
            for (int k = 12; k < 16; k++) hs[k] = 0u;
        }
    }
#pragma unroll
    for (int k = 0; k < 16; k++) K[k] = hs[k];
    bs = 32u + 16u * hsel;
    r6_store_k(S, len, bs, K, colbytes);
    return prev[3] & 0xffu;
}

/* Slots and classes.  One workgroup per CU (12 waves) holds up to R6_MAX_SLOTS candidates ("slots") --
 * more slots than lanes; everything a slot needs between rounds is in LDS: its period (pw || K[0:bs] ||
 * wrap) in a column of a pattern area, a state word and its candidate number.  A round costs
 * 64 x (len + bs) bytes of AES-CBC + a SHA-256 or SHA-384/512 pass over them, and the family is only known
 * after the round's first ciphertext block, so a wave runs a round for 64 slots of ONE class
 * (class = (family is SHA-256 ? 0 : 3) + (bs - 32) / 16: same hash code, same trip count).
 *
 * Flow scheduling, no barriers: a slot that finishes its round (or starts a candidate) computes the family
 * of its next round (one AES block) and is queued in its class's bitmap; a wave that is free claims up to
 * 64 queued slots of the fullest class (bitmap words, atomicAnd) and runs one round of them.  Waves
 * never wait for each other.  The previous schedule -- all slots sorted per interval, batches listed
 * costliest first, a workgroup barrier per interval -- left 16 % of wave time at the barriers
 * (a round-2 per-wave cycle count): ~20 batches of 1-2 M cycles over 12 waves leave a long tail every interval.
 *
 * Deadlock freedom (the round-1 lock-based queue hung): there is no lock and no wave ever waits on a value
 * only another waiting wave could produce.  Every claim is one wave-uniform pass (lane 0's decisions
 * broadcast by readfirstlane), so no lane of a wave spins while another lane of the same wave holds
 * something; a wave that finds nothing queued sleeps and re-reads (atomic loads, never hoisted) only while
 * `live` > 0, i.e. while some other wave is running a round whose slots it will queue or retire.  `live`
 * (slots holding a candidate) only falls when a slot finds the launch's cursor exhausted; at 0 every wave
 * leaves the loop, and the grid drains.
 *
 * Pattern areas: the dynamic area holds slots in groups of 64 (column 4*(slot%64)); when the tables take only
 * half of each row (R6_TE_USED <= 128, not the default) slots [0, te_slots) live in the free upper halves in
 * groups of 32 (column 128 + 4*(slot%32)).  Rows are 256 bytes apart in both, so r6_read16 and friends see
 * one layout. */
#ifndef R6_LANES
#define R6_LANES 768
#endif
#ifndef R6_MAX_SLOTS
#define R6_MAX_SLOTS 1088           /* 17 groups: the slot arrays sized so that 16 groups of 21-word columns fit */
#endif
#define R6_SLOTS_PER_THREAD ((R6_MAX_SLOTS + R6_LANES - 1) / R6_LANES)
#define R6_CLASSES 6
#define R6_QUEUES R6_CLASSES
#define R6_MAP_WORDS ((R6_MAX_SLOTS + 31) / 32)
#define R6_IDLE 0xffffffffu
#ifndef R6_WATCHDOG_S
#define R6_WATCHDOG_S 10u           /* seconds a wave may find nothing queued while slots are live */
#endif

struct r6_shared {
    uint32_t map[R6_QUEUES][R6_MAP_WORDS];    /* queued slots of each class, a bit per slot */
    uint32_t count[R6_QUEUES];                /* queued slots per queue (a hint for picking one)       */
    uint32_t live;                            /* slots holding a candidate                             */
    uint32_t nslots, te_slots, ncand, pat_words;
    const uint32_t *slots;                    /* e.slots, e.lens (list mode), likewise */
    const uint8_t *lens;
    const uint64_t *loff;                     /* e.loff, e.llen, e.keys (long list mode) */
    const uint32_t *llen;
    const uint32_t *keys;
    unsigned long long start;                 /* e.start / e.count (ncand) read from here when a slot takes or reports a
                                                 candidate: kept in registers across the persistent loop, the
                                                 64-bit start was spilled to scratch (SGPR pressure) */
    uint8_t sdig[DPRF_MAX_RANGE_LEN];         /* base-cslen digits of the launch's first index          */
    uint16_t stage[R6_LANES / 64][64];        /* per wave: the slot ids of the batch it claimed         */
    unsigned long long idle_t0[R6_LANES / 64];  /* per wave: wall clock when it first found nothing queued, 0 while
                                                 it finds work (in LDS: a 64-bit value held in registers across the
                                                 loop was one of the split-AES build's spills) */
    uint32_t state[R6_MAX_SLOTS];             /* len | bs << 8 | round << 16                            */
    uint32_t cand[R6_MAX_SLOTS];              /* candidate offset within the launch, R6_IDLE when none  */
};

DEVI r6_lds slot_lds(uint32_t patbase, uint32_t pat_words, uint32_t te_slots, uint32_t slot, uint32_t lane) {
    r6_lds S;
    if (slot < te_slots) {                  /* only when the tables leave the upper half of each row */
        S.pat = lds_addr(r6_te) + (slot >> 5) * pat_words * 256u;
        S.lanebase = 128u + ((slot & 31u) << 2);
    } else {
        const uint32_t t = slot - te_slots;
        S.pat = patbase + (t >> 6) * pat_words * 256u;
        S.lanebase = (t & 63u) << 2;
    }
    S.lanec = (lane & (R6_TE_COPIES - 1u)) << 2;
    /* copy c = lane % 16 in every byte; table offsets 64 t: A (lane bit 4 clear) T_t / B T_t+1 for lookup t */
    const uint32_t c4 = S.lanec * 0x01010101u;
    const bool gb = (lane & 16u) != 0u;
    S.base = c4 + (gb ? 0x00c08040u : 0xc0804000u);
    return S;
}

DEVI uint32_t lds_load(const uint32_t *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
DEVI unsigned long long lds_load64(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

/* Candidate numbers for the active lanes that ask (need): ONE atomicAdd on the launch's cursor per wave, each
 * asking lane gets base + its rank among them (ids stay in increasing lane order).  A per-lane atomic made every
 * candidate start a device-scope atomic: ~31 B of HBM writes per candidate (profiles/prof_pdf_r6_r03a.json). */
DEVI uint32_t r6_take(dprf_results *R, bool need, uint32_t lane) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(need);
    if (m == 0) return R6_IDLE;
    const uint32_t leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(&R->cursor, (uint32_t)__builtin_popcountll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    return need ? base + rank : R6_IDLE;
}

/* Start candidate c (from r6_take) in `slot`; false when there is none (cursor exhausted, or skipped under
 * stop_on_first). */
template <int MODE>
DEVI bool r6_start(const dprf_enum &e, const dprf_pdf_params &p, const uint8_t *cs, dprf_results *R,
                   uint32_t stop_on_first, r6_shared *sh, const r6_lds &S, uint32_t slot, uint32_t c) {
    /* the cursor hands out candidates in increasing order, so every candidate below one that is taken has
     * been taken and will finish: skipping those above the lowest hit so far (stop_on_first) keeps the
     * reported hit the lowest of the call */
    if (c >= lds_load(&sh->ncand)) {
        c = R6_IDLE;
    } else if (stop_on_first && lds_load64(&sh->start) + c > lowest_known(e, R)) {
        atomicAdd(&R->skipped, 1ull);
        c = R6_IDLE;
    }
    sh->cand[slot] = c;
    if (c == R6_IDLE) return false;
    uint32_t K[16];
    const uint32_t len = r6_begin<MODE>(e, p, cs, sh->sdig, lds_load64(&sh->start) + c, c, sh->slots, sh->lens, S, K,
                                        sh->loff, sh->llen, sh->keys, lds_load(&sh->ncand));
    r6_store_k(S, len, 32u, K, MODE == 0 ? 4u * lds_load(&sh->pat_words) : ~0u);   /* list mode: full wrap */
    sh->state[slot] = len | (32u << 8);
    return true;
}

/* Queue a slot holding a candidate in the class of its next round. */
DEVI void r6_push(r6_shared *sh, const r6_lds &S, uint32_t slot) {
    const uint32_t st = sh->state[slot];
    const uint32_t fam = r6_family(S, st & 0xffu);
    const uint32_t cls = (fam ? 3u : 0u) + (((st >> 8) & 0xffu) - 32u) / 16u;
    sh->state[slot] = (st & 0x3fffffffu) | (fam << 30);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");         /* state/period before the bit */
    atomicOr(&sh->map[cls][slot >> 5], 1u << (slot & 31u));
    atomicAdd(&sh->count[cls], 1u);
}


/* Wave-uniform: claim up to 64 queued slots of the fullest class; returns how many (0: none queued) and
 * this lane's slot in *slot.  Lane w < R6_MAP_WORDS owns bitmap word w; lanes take their words' bits in
 * order up to 64 in total, clear exactly the bits they chose (atomicAnd returns what they got when another
 * wave raced them), and the ids are handed out through the wave's stage row. */
template <int MODE>
DEVI uint32_t r6_claim(r6_shared *sh, uint32_t lane, uint32_t wave, uint32_t *slot) {
    const uint32_t cnt = lane < R6_QUEUES ? lds_load(&sh->count[lane]) : 0u;
    uint32_t best = R6_CLASSES, bc = 0;
#pragma unroll
    for (int c = 0; c < R6_CLASSES; c++) {
        const uint32_t v = __builtin_amdgcn_readlane(cnt, c);
        if (v > bc) { bc = v; best = c; }
    }
    if (bc == 0) return 0;
    const uint32_t w = lane < R6_MAP_WORDS ? lds_load(&sh->map[best][lane]) : 0u;
    const uint32_t pc = __builtin_popcount(w);
    /* inclusive scan of the word popcounts over the wave */
    uint32_t inc = pc;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += o;
    }
    /* whole words while the running total stays <= 64; the word that crosses 64 gives its lowest bits */
    uint32_t take = 0u;
    if (inc <= 64u) {
        take = w;
    } else if (inc - pc < 64u) {
        for (uint32_t k = 64u - (inc - pc), rest = w; k; k--) {
            take |= rest & (0u - rest);
            rest &= rest - 1u;
        }
    }
    const uint32_t got = take ? (atomicAnd(&sh->map[best][lane], ~take) & take) : 0u;
    /* ids packed densely in claim order.  Measured and dropped (round 3): placing each slot id on lane id % 64 so that
     * the lanes of one 32-lane LDS access group hit distinct period-column banks -- conflicts 3.4 -> 3.0 % of the CU
     * cycles, but 3.50 -> 3.46 M cand/s for the extra scans */
    const uint32_t ng = __builtin_popcount(got);
    uint32_t off = ng;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(off, d, 64);
        if (lane >= (uint32_t)d) off += o;
    }
    const uint32_t total = __builtin_amdgcn_readlane(off, 63);
    off -= ng;
    for (uint32_t b = got; b; b &= b - 1u) sh->stage[wave][off++] = (uint16_t)(lane * 32u + __builtin_ctz(b));
    if (lane == 0 && total) atomicSub(&sh->count[best], total);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");       /* stage writes -> reads; bits -> slot state */
    *slot = lane < total ? sh->stage[wave][lane] : R6_IDLE;
    return total;
}

template <int MODE>
__global__ void __launch_bounds__(R6_LANES, 1)     /* 12 waves/CU: <= 168 VGPRs */
k_pdf_r6(dprf_enum e, dprf_pdf_params p, const dprf_aes_tables *T, dprf_results *R, uint32_t cap,
         uint32_t stop_on_first, uint32_t pat_words, uint32_t nslots, uint32_t te_slots, uint64_t idle_ticks) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];               /* after r6_te */
    uint8_t *cs = (uint8_t *)smem;                                              /* 256 B */
    r6_shared *sh = (r6_shared *)((uint8_t *)smem + 256);
    const uint32_t patbase = lds_addr(smem) + 256u + (uint32_t)((sizeof(r6_shared) + 15) / 16 * 16);
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, nthr = blockDim.x;
    /* the asm rounds use the v_perm result as the whole LDS address: r6_te must sit at LDS address 0 (it is this
     * kernel's only static LDS object).  A build that ever breaks this fails loudly instead of computing wrong. */
    if (lds_addr(r6_te) != 0u) {
        if (tid == 0) atomicOr(&R->pad_, 8u);
        return;
    }
    /* the tables' copies fill each row: table t = ror(Te0, 8t) */
    constexpr uint32_t TW = R6_TE_USED / 4;                                     /* table words per row */
    for (uint32_t k = tid; k < 256u * TW; k += nthr) {
        const uint32_t x = k / TW, c = k % TW, t = c / R6_TE_COPIES;
        r6_te[x * (R6_TE_ROW_BYTES / 4) + c] = ror32(T->te0[x], 8 * t);
    }
    for (uint32_t k = tid; k < 64; k += nthr) ((uint32_t *)cs)[k] = ((const uint32_t *)e.charset)[k];
    for (uint32_t k = tid; k < R6_QUEUES * R6_MAP_WORDS; k += nthr) (&sh->map[0][0])[k] = 0u;
    if (tid < R6_QUEUES) sh->count[tid] = 0u;
    if (tid < DPRF_MAX_RANGE_LEN) sh->sdig[tid] = e.sdig[tid];
    if (tid == 0) {
        sh->live = 0u;
        sh->start = e.start;
        sh->ncand = e.count;
        sh->pat_words = pat_words;
        sh->slots = e.slots;
        sh->lens = e.lens;
        sh->loff = e.loff;
        sh->llen = e.llen;
        sh->keys = e.keys;
    }
    __syncthreads();

    for (uint32_t sl = tid; sl < nslots; sl += nthr) {
        const r6_lds S = slot_lds(patbase, pat_words, te_slots, sl, lane);
        if (r6_start<MODE>(e, p, cs, R, stop_on_first, sh, S, sl, r6_take(R, true, lane))) {
            atomicAdd(&sh->live, 1u);
            r6_push(sh, S, sl);
        }
    }
    __syncthreads();
    if (lane == 0) sh->idle_t0[wave] = 0ull;
    for (;;) {
        uint32_t slot;
        const uint32_t n = r6_claim<MODE>(sh, opaque_lane(), wave, &slot);
        if (n == 0) {
            if (lds_load(&sh->live) == 0u) break;                  /* uniform: one LDS word */
            /* watchdog on the constant-rate wall clock: a wave that has found nothing queued for idle_ticks
             * (host: 10 s; a whole launch is ~3 s and the drain after the cursor runs dry tens of ms) gives up
             * and flags the launch instead of hanging the device; the host turns the flag into an error */
            const uint64_t now = wall_clock64() | 1ull;                 /* never 0: 0 marks "not idling" */
            const unsigned long long t0 = lds_load64(&sh->idle_t0[wave]);
            if (t0 == 0ull) {
                if (lane == 0) __hip_atomic_store(&sh->idle_t0[wave], (unsigned long long)now, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_WORKGROUP);
            } else if (now - t0 > idle_ticks) {
                if (lane == 0) atomicOr(&R->pad_, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(4);
            continue;
        }
        if (lane == 0) __hip_atomic_store(&sh->idle_t0[wave], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (slot != R6_IDLE) {
            const r6_lds S = slot_lds(patbase, pat_words, te_slots, slot, opaque_lane());
            const uint32_t st = sh->state[slot];
            const uint32_t len = st & 0xffu, hs = st >> 30;
            uint32_t bs = (st >> 8) & 0xffu, i = (st >> 16) & 0x3fffu;
            uint32_t K[16];
            const uint32_t last = r6_round<MODE == 0>(S, len, bs, hs, K, MODE == 0 ? 4u * lds_load(&sh->pat_words) : ~0u);
            i++;
            bool more = true;
            if (i >= 64u && i >= last + 32u) {                    /* loop condition of :247 */
                bool ok = true;
#pragma unroll
                for (int kk = 0; kk < 8; kk++) ok = ok && K[kk] == p.u[kk];
                if (ok) report_hit(e, R, lds_load64(&sh->start) + sh->cand[slot], cap, stop_on_first);
                /* the finishing lanes of the batch take their next candidates together */
                more = r6_start<MODE>(e, p, cs, R, stop_on_first, sh, S, slot, r6_take(R, true, opaque_lane()));
                if (!more) atomicSub(&sh->live, 1u);
            } else {
                sh->state[slot] = len | (bs << 8) | (i << 16);
            }
            if (more) r6_push(sh, S, slot);
        }
    }
}

/* Slot capacity of one workgroup: 32-slot groups in the upper halves of the Te0 rows, then 64-slot groups
 * in the dynamic LDS left next to the table and the shared block (160 KiB per workgroup). */
/* -pr 6 (21-word columns, r6_pat_words): 16 groups of 64 slots beside the tables and the shared block */
static_assert(R6_TE_BYTES + 256 + (sizeof(r6_shared) + 15) / 16 * 16 + 16 * 21 * 256 <= 160 * 1024, "16 groups at -pr 6");
static void r6_capacity(uint32_t pat_words, uint32_t *nslots, uint32_t *te_slots, size_t *shm) {
    const size_t fixed = R6_TE_BYTES + 256 + (sizeof(r6_shared) + 15) / 16 * 16;
    const uint32_t te_groups = R6_TE_USED <= 128 ? 256u / pat_words : 0u;
    uint32_t te = te_groups * 32u;
    uint32_t dyn = (uint32_t)((160u * 1024u - fixed) / ((size_t)pat_words * 256u)) * 64u;
    if (te > R6_MAX_SLOTS) te = R6_MAX_SLOTS;
    if (te + dyn > R6_MAX_SLOTS) dyn = (R6_MAX_SLOTS - te) / 64u * 64u;
    *te_slots = te;
    *nslots = te + dyn;
    *shm = 256 + (sizeof(r6_shared) + 15) / 16 * 16 + (size_t)(dyn / 64u) * pat_words * 256u;   /* + static r6_te */
}

/* Words per period column.  List mode: the period (lmax + 64) + 16 wrap bytes and the fifth word of any block read
 * (r6_read16 takes 5 words from word o / 4).  Range mode: exactly the words the reads reach -- the block of a round
 * starts at o = 16 q mod Lp (Lp = lmax + bs, so o runs over the multiples of gcd(16, Lp)) and takes 4 words, 5 when
 * o is not a word start; r6_load_k reads 5 words from bytes lmax and lmax + 16.  Even password lengths then need one
 * word less (21 instead of 22 at -pr 6: 1,024 slots per CU instead of 960). */
static uint32_t r6_pat_words(uint32_t mode, uint32_t lmax) {
    if (mode != 0) return ((lmax + 63u) >> 2) + 5u;
    uint32_t mx = ((lmax + 16u) >> 2) + 5u;
    for (uint32_t bs = 32; bs <= 64; bs += 16) {
        const uint32_t Lp = lmax + bs;
        uint32_t g = 16;
        while (Lp % g) g >>= 1;
        for (uint32_t o = 0; o < Lp; o += g) {
            const uint32_t w = (o >> 2) + ((o & 3u) ? 5u : 4u);
            if (w > mx) mx = w;
        }
    }
    return mx;
}

#define R6_MAX_DEVICES 64
static std::mutex r6_attr_mu;
static bool r6_attr_set[3][R6_MAX_DEVICES];

hipError_t launch_pdf_r6(const dprf_enum &e, const dprf_pdf_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s) {
    /* longest password of the launch (list mode: the host's maximum over the chunk): the period length
     * and with it the slots per CU follow the actual candidates, not the 64-byte slot width */
    const uint32_t lcap = e.mode == 2 ? (uint32_t)DPRF_R6_MAX_LONG : 4u * DPRF_SLOT_WORDS;
    const uint32_t lmax = e.pwlen < lcap ? e.pwlen : lcap;
    const uint32_t pat_words = r6_pat_words(e.mode, lmax);
    uint32_t nslots = 0, te_slots = 0;
    size_t shm = 0;
    r6_capacity(pat_words, &nslots, &te_slots, &shm);
    if (nslots < 64) return hipErrorInvalidValue;
    /* lanes: 12 waves, or fewer when there are fewer slots */
    uint32_t lanes = (nslots / 64u) * 64u;
    if (lanes > R6_LANES) lanes = R6_LANES;
    /* the work cursor restarts at 0 for every launch (stream-ordered before the kernel) */
    hipError_t me = hipMemsetAsync(&R->cursor, 0, sizeof(uint32_t), s);
    if (me != hipSuccess) return me;
    int dev = 0, ncu = 0;
    if ((me = hipGetDevice(&dev)) != hipSuccess) return me;
    if (dev < 0 || dev >= R6_MAX_DEVICES) return hipErrorInvalidDevice;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
    int clk_khz = 0;                                              /* wall_clock64() rate (100 MHz on gfx9) */
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, dev);
    if (clk_khz <= 0) clk_khz = 100000;
    const uint64_t idle_ticks = (uint64_t)clk_khz * 1000u * R6_WATCHDOG_S;
    /* one workgroup per CU; a launch smaller than the slots it would open uses fewer workgroups */
    uint32_t grid = (e.count + nslots - 1) / nslots;
    if (grid > (uint32_t)ncu) grid = (uint32_t)ncu;
    const void *fn = e.mode == 0 ? (const void *)k_pdf_r6<0> : e.mode == 1 ? (const void *)k_pdf_r6<1>
                                                                            : (const void *)k_pdf_r6<2>;
    {
        /* function attributes are per device: set once per (device, mode), under a lock -- the device
         * workers of a multi-device context launch concurrently */
        std::lock_guard<std::mutex> g(r6_attr_mu);
        bool &done = r6_attr_set[e.mode < 3 ? e.mode : 2][dev];
        if (!done) {
            me = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - R6_TE_BYTES);
            if (me != hipSuccess) return me;
            done = true;
        }
    }
    if (e.mode == 0)
        hipLaunchKernelGGL(k_pdf_r6<0>, dim3(grid), dim3(lanes), shm, s, e, p, T, R, cap, stop, pat_words, nslots,
                           te_slots, idle_ticks);
    else if (e.mode == 1)
        hipLaunchKernelGGL(k_pdf_r6<1>, dim3(grid), dim3(lanes), shm, s, e, p, T, R, cap, stop, pat_words, nslots,
                           te_slots, idle_ticks);
    else
        hipLaunchKernelGGL(k_pdf_r6<2>, dim3(grid), dim3(lanes), shm, s, e, p, T, R, cap, stop, pat_words, nslots,
                           te_slots, idle_ticks);
    return hipGetLastError();
}

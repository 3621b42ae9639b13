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
 *  - AES T-table: Te0 only (Te1..3 by rotation), replicated 16x across banks (entry x of copy c at
 *    word 16x+c, lane l reads copy l%16) -- random table indices otherwise pile up on few banks
 *    (measured 1.5x, tools/aes_lds_bench.hip).  The last round takes S[x] from byte 2 of Te0[x].
 *  - Persistent lanes: a wave owns a contiguous range of candidates; a lane that finishes its
 *    candidate (after 64..~110 rounds) immediately takes the next one, so the wave never idles on its
 *    slowest lane until the range is exhausted.
 *  - The hash family is chosen per lane after the first ciphertext block; a wave runs the SHA-256 and
 *    SHA-512 paths predicated.
 */
#include "dev_crypto.h"
#include "dprf_params.h"
#include "dprf_launch.h"

#define R6_TE_COPIES 16
#define R6_PER_LANE 4           /* candidates per lane per launch (persistent refill) */

DEVI uint32_t fastdiv6(uint32_t n, uint32_t m, uint32_t s) {
    uint32_t t = __umulhi(n, m);
    return (t + ((n - t) >> 1)) >> s;
}

struct r6_lds {
    const uint32_t *te;        /* R6_TE_COPIES x 256 words */
    uint8_t *pat;              /* [pat_words][64 lanes] words for this wave */
    uint32_t lanebase;         /* lane * 4 */
    uint32_t tebase;           /* (lane % 16) */
};

DEVI uint32_t te_(const r6_lds &S, uint32_t x) { return S.te[(x << 4) | S.tebase]; }
DEVI uint32_t pat_addr(uint32_t pos, uint32_t lanebase) { return ((pos >> 2) << 8) | (pos & 3u) | lanebase; }

DEVI void aes128_expand_te(const r6_lds &S, const uint32_t key[4], uint32_t rk[44]) {
    const uint32_t rcon[10] = {0x01000000u, 0x02000000u, 0x04000000u, 0x08000000u, 0x10000000u,
                               0x20000000u, 0x40000000u, 0x80000000u, 0x1b000000u, 0x36000000u};
    rk[0] = key[0]; rk[1] = key[1]; rk[2] = key[2]; rk[3] = key[3];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        const uint32_t t = rk[4 * i + 3];
        /* SubWord(RotWord(t)) with S[x] = byte 2 of Te0[x] */
        const uint32_t sw = ((te_(S, B2(t)) << 8) & 0xff000000u) | (te_(S, B1(t)) & 0x00ff0000u) |
                            ((te_(S, B0(t)) >> 8) & 0x0000ff00u) | ((te_(S, B3(t)) >> 16) & 0xffu);
        rk[4 * i + 4] = rk[4 * i] ^ sw ^ rcon[i];
        rk[4 * i + 5] = rk[4 * i + 1] ^ rk[4 * i + 4];
        rk[4 * i + 6] = rk[4 * i + 2] ^ rk[4 * i + 5];
        rk[4 * i + 7] = rk[4 * i + 3] ^ rk[4 * i + 6];
    }
}

DEVI void aes128_encrypt_te(const r6_lds &S, const uint32_t rk[44], uint32_t s0, uint32_t s1, uint32_t s2,
                            uint32_t s3, uint32_t out[4]) {
    s0 ^= rk[0]; s1 ^= rk[1]; s2 ^= rk[2]; s3 ^= rk[3];
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const uint32_t t0 = xor3(xor3(te_(S, B3(s0)), ror32(te_(S, B2(s1)), 8), ror32(te_(S, B1(s2)), 16)),
                                 ror32(te_(S, B0(s3)), 24), rk[4 * r]);
        const uint32_t t1 = xor3(xor3(te_(S, B3(s1)), ror32(te_(S, B2(s2)), 8), ror32(te_(S, B1(s3)), 16)),
                                 ror32(te_(S, B0(s0)), 24), rk[4 * r + 1]);
        const uint32_t t2 = xor3(xor3(te_(S, B3(s2)), ror32(te_(S, B2(s3)), 8), ror32(te_(S, B1(s0)), 16)),
                                 ror32(te_(S, B0(s1)), 24), rk[4 * r + 2]);
        const uint32_t t3 = xor3(xor3(te_(S, B3(s3)), ror32(te_(S, B2(s0)), 8), ror32(te_(S, B1(s1)), 16)),
                                 ror32(te_(S, B0(s2)), 24), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    /* last round: SubBytes + ShiftRows + AddRoundKey, S[x] = byte 2 of Te0[x] */
#define SB3(x) ((te_(S, (x)) << 8) & 0xff000000u)
#define SB2(x) (te_(S, (x)) & 0x00ff0000u)
#define SB1(x) ((te_(S, (x)) >> 8) & 0x0000ff00u)
#define SB0(x) ((te_(S, (x)) >> 16) & 0x000000ffu)
    out[0] = (SB3(B3(s0)) | SB2(B2(s1)) | SB1(B1(s2)) | SB0(B0(s3))) ^ rk[40];
    out[1] = (SB3(B3(s1)) | SB2(B2(s2)) | SB1(B1(s3)) | SB0(B0(s0))) ^ rk[41];
    out[2] = (SB3(B3(s2)) | SB2(B2(s3)) | SB1(B1(s0)) | SB0(B0(s1))) ^ rk[42];
    out[3] = (SB3(B3(s3)) | SB2(B2(s0)) | SB1(B1(s1)) | SB0(B0(s2))) ^ rk[43];
#undef SB3
#undef SB2
#undef SB1
#undef SB0
}

/* SHA-512 over 32 BE words held as two 16-word halves; state as 16 BE words (hi, lo pairs) */
DEVI void sha512_compress_pairs(uint32_t hs[16], const uint32_t lo[16], const uint32_t hi[16]) {
    uint64_t st[8], w[16];
#pragma unroll
    for (int k = 0; k < 8; k++) st[k] = ((uint64_t)hs[2 * k] << 32) | hs[2 * k + 1];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = ((uint64_t)lo[2 * k] << 32) | lo[2 * k + 1];
#pragma unroll
    for (int k = 0; k < 8; k++) w[8 + k] = ((uint64_t)hi[2 * k] << 32) | hi[2 * k + 1];
    sha512_compress(st, w);
#pragma unroll
    for (int k = 0; k < 8; k++) { hs[2 * k] = (uint32_t)(st[k] >> 32); hs[2 * k + 1] = (uint32_t)st[k]; }
}

/* Load candidate `idx` (keyspace index or slot), compute K = SHA256(pw || salt), write pw to the
 * head of the lane's pattern column.  Returns the password length. */
template <int MODE>
DEVI uint32_t r6_begin(const dprf_enum &e, const dprf_pdf_params &p, const uint8_t *cs, uint64_t idx,
                       const r6_lds &S, uint32_t K[16]) {
    uint32_t w[DPRF_SLOT_WORDS];
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) w[j] = 0;
    uint32_t len;
    if (MODE == 0) {
        uint32_t rem = (uint32_t)(idx - e.start), carry = 0;
#pragma unroll
        for (int pp = DPRF_MAX_RANGE_LEN - 1; pp >= 0; --pp) {
            if ((uint32_t)pp < e.pwlen) {
                uint32_t q = e.cslen == 1 ? rem : fastdiv6(rem, e.div_m, e.div_s);
                uint32_t r = rem - q * e.cslen;
                uint32_t d = (uint32_t)e.sdig[pp] + r + carry;
                carry = d >= e.cslen ? 1u : 0u;
                d -= carry ? e.cslen : 0u;
                rem = q;
                w[pp >> 2] |= (uint32_t)cs[d] << (8 * (pp & 3));
            }
        }
        len = e.pwlen;
    } else {
        const uint4 *s = (const uint4 *)(e.slots + idx * DPRF_SLOT_WORDS);
#pragma unroll
        for (int q = 0; q < DPRF_SLOT_WORDS / 4; q++) {
            uint4 v = s[q];
            w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
        }
        len = e.lens[idx];
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
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) *(uint32_t *)(S.pat + (((uint32_t)j << 8) | S.lanebase)) = w[j];
    return len;
}

/* One round of the hardened hash for this lane: K, bs updated; returns E[last]. */
DEVI uint32_t r6_round(const r6_lds &S, uint32_t len, uint32_t &bs, uint32_t K[16]) {
    const uint32_t Lp = len + bs;
    /* period = pw || K[0:bs], then its first 16 bytes again (a 16-byte read at o < Lp never wraps) */
#pragma unroll
    for (int k = 0; k < 64; k++) {
        if ((uint32_t)k < bs) {
            const uint32_t b = (K[k >> 2] >> (24 - 8 * (k & 3))) & 0xffu;
            S.pat[pat_addr(len + k, S.lanebase)] = (uint8_t)b;
        }
    }
    for (uint32_t k = 0; k < 16; k++) S.pat[pat_addr(Lp + k, S.lanebase)] = S.pat[pat_addr(k, S.lanebase)];
    /* AES-128 key K[0:16], iv K[16:32] (:259-261) */
    uint32_t rk[44];
    aes128_expand_te(S, K, rk);
    uint32_t prev[4] = {K[4], K[5], K[6], K[7]};
    uint32_t hs[16], half[16];
    uint32_t hsel = 0;          /* 0: SHA-256, 1: SHA-384, 2: SHA-512 */
    uint32_t o = 0;
    for (uint32_t u = 0; u < Lp; u++) {         /* 64-byte units; per-lane trip count */
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t wi = o >> 2;
            const uint32_t sel = 0x00010203u + (o & 3u) * 0x01010101u;
            const uint32_t *col = (const uint32_t *)(S.pat + ((wi << 8) | S.lanebase));
            uint32_t lw[5];
#pragma unroll
            for (int k = 0; k < 5; k++) lw[k] = col[k * 64];
            uint32_t y[4];
            aes128_encrypt_te(S, rk, perm(lw[1], lw[0], sel) ^ prev[0], perm(lw[2], lw[1], sel) ^ prev[1],
                              perm(lw[3], lw[2], sel) ^ prev[2], perm(lw[4], lw[3], sel) ^ prev[3], y);
#pragma unroll
            for (int k = 0; k < 4; k++) { prev[k] = y[k]; w[4 * q + k] = y[k]; }
            o += 16u;
            o = o >= Lp ? o - Lp : o;
            if (q == 0 && u == 0) {
                /* Step 4: SHA-2 size from sum(E[0:16]) mod 3 (:264-268) */
                uint32_t sum = __builtin_amdgcn_sad_u8(y[0], 0u, 0u);
                sum = __builtin_amdgcn_sad_u8(y[1], 0u, sum);
                sum = __builtin_amdgcn_sad_u8(y[2], 0u, sum);
                sum = __builtin_amdgcn_sad_u8(y[3], 0u, sum);
                hsel = sum % 3u;
                if (hsel == 0) {
                    sha256_iv(hs);
                } else {
                    uint64_t iv[8];
                    sha512_iv(iv, hsel == 1);
#pragma unroll
                    for (int k = 0; k < 8; k++) { hs[2 * k] = (uint32_t)(iv[k] >> 32); hs[2 * k + 1] = (uint32_t)iv[k]; }
                }
            }
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
    if (hsel == 0) {
        uint32_t w[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
        sha256_compress(hs, w);
#pragma unroll
        for (int k = 8; k < 16; k++) hs[k] = 0u;
    } else {
        uint32_t w[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
        if (Lp & 1u) {
            sha512_compress_pairs(hs, half, w);
        } else {
            uint32_t z[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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
    return prev[3] & 0xffu;
}

template <int MODE>
__global__ void __launch_bounds__(256, 3)     /* <= 168 VGPRs: 3 waves/SIMD; the unit loop stays spill-free */
k_pdf_r6(dprf_enum e, dprf_pdf_params p, const dprf_aes_tables *T, dprf_results *R, uint32_t cap,
         uint32_t stop_on_first, uint32_t pat_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    uint32_t *te = smem;                                                   /* 16 KiB */
    uint8_t *cs = (uint8_t *)(smem + R6_TE_COPIES * 256);                  /* 256 B */
    uint32_t *flag = smem + R6_TE_COPIES * 256 + 64;
    uint8_t *patbase = (uint8_t *)(smem + R6_TE_COPIES * 256 + 64 + 4);    /* 4 waves x pat_words x 256 B */
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < R6_TE_COPIES * 256; k += blockDim.x) te[k] = T->te0[k / R6_TE_COPIES];
    for (uint32_t k = tid; k < 64; k += blockDim.x) ((uint32_t *)cs)[k] = ((const uint32_t *)e.charset)[k];
    if (tid == 0) *flag = stop_on_first ? __hip_atomic_load(&R->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    __syncthreads();
    if (*flag) return;

    const uint32_t lane = tid & 63u, wave = tid >> 6;
    r6_lds S;
    S.te = te;
    S.pat = patbase + (size_t)wave * pat_words * 256u;
    S.lanebase = lane << 2;
    S.tebase = lane & (R6_TE_COPIES - 1);

    /* this wave's contiguous range of candidates (offsets within the launch) */
    const uint32_t per_wave = 64u * R6_PER_LANE;
    const uint32_t wbeg = (blockIdx.x * (blockDim.x >> 6) + wave) * per_wave;
    const uint32_t wend = min(wbeg + per_wave, e.count);
    uint32_t next = wbeg + 64u;                  /* wave-uniform: next unassigned offset */
    uint32_t mine = wbeg + lane;
    bool act = mine < wend;
    uint32_t K[16], len = 0, bs = 32, i = 0;
    if (act) len = r6_begin<MODE>(e, p, cs, e.start + mine, S, K);
    while (__any(act)) {
        bool fin = false;
        if (act) {
            const uint32_t last = r6_round(S, len, bs, K);
            i++;
            fin = i >= 64u && i >= last + 32u;          /* loop condition of :247 */
            if (fin) {
                bool ok = true;
#pragma unroll
                for (int k = 0; k < 8; k++) ok = ok && K[k] == p.u[k];
                if (ok) {
                    const unsigned long long idx = e.start + mine;
                    uint32_t slot = atomicAdd(&R->nhits, 1u);
                    if (slot < cap) R->hits[slot] = idx;
                    atomicMin(&R->first, idx);
                    if (stop_on_first) atomicExch(&R->stop, 1u);
                }
            }
        }
        /* refill finished lanes with the wave's next candidates */
        const unsigned long long m = __ballot(fin);
        if (fin) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            mine = next + rank;
            act = mine < wend;
            if (act) { bs = 32; i = 0; len = r6_begin<MODE>(e, p, cs, e.start + mine, S, K); }
        }
        next += (uint32_t)__popcll(m);
    }
    if (lane == 0 && wbeg < e.count) atomicAdd(&R->evaluated, (unsigned long long)(wend - wbeg));
}

hipError_t launch_pdf_r6(const dprf_enum &e, const dprf_pdf_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s) {
    const uint32_t lmax = e.mode == 0 ? e.pwlen : 4u * DPRF_SLOT_WORDS;
    /* period (lmax + 64) + 16 wrap bytes, + 4 words read past the last block start */
    const uint32_t pat_words = (lmax + 64u + 16u + 3u) / 4u + 1u;
    const size_t shm = (size_t)R6_TE_COPIES * 1024u + 256u + 16u + 4u * (size_t)pat_words * 256u;
    static bool attr_set[2] = {false, false};
    const uint32_t per_block = 4u * 64u * R6_PER_LANE;
    dim3 grid((e.count + per_block - 1) / per_block);
    if (e.mode == 0) {
        if (!attr_set[0]) { (void)hipFuncSetAttribute((const void *)k_pdf_r6<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); attr_set[0] = true; }
        hipLaunchKernelGGL(k_pdf_r6<0>, grid, dim3(256), shm, s, e, p, T, R, cap, stop, pat_words);
    } else {
        if (!attr_set[1]) { (void)hipFuncSetAttribute((const void *)k_pdf_r6<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); attr_set[1] = true; }
        hipLaunchKernelGGL(k_pdf_r6<1>, grid, dim3(256), shm, s, e, p, T, R, cap, stop, pat_words);
    }
    return hipGetLastError();
}

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
 * `data` is never materialised: each lane keeps ONE doubled copy of its period (pw || K[0:bs]) in its
 * own LDS bank column and streams 16-byte blocks out of it with one v_perm per word; ciphertext goes
 * straight into the SHA message registers 64 bytes (4 AES blocks) at a time.  The hash choice is per
 * lane (known after the first AES block), so a wave runs the SHA-256 and SHA-512 paths predicated;
 * lanes that finish early idle until the wave's last lane is done.
 */
#include "dev_crypto.h"
#include "dprf_params.h"
#include "dprf_launch.h"

struct cand6 {
    uint32_t w[DPRF_SLOT_WORDS];
    uint32_t len;
};

DEVI uint32_t fastdiv6(uint32_t n, uint32_t m, uint32_t s) {
    uint32_t t = __umulhi(n, m);
    return (t + ((n - t) >> 1)) >> s;
}

/* byte address of pattern byte `pos` of this lane: word (pos>>2) of a [word][64 lanes] column layout */
DEVI uint32_t pat_addr(uint32_t pos, uint32_t lanebase) {
    return ((pos >> 2) << 8) | (pos & 3u) | lanebase;
}

/* 64-bit SHA-512 compression over 32 BE 32-bit words */
DEVI void sha512_compress_w32(uint64_t st[8], const uint32_t lo[16], const uint32_t hi[16]) {
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = ((uint64_t)lo[2 * k] << 32) | lo[2 * k + 1];
#pragma unroll
    for (int k = 0; k < 8; k++) w[8 + k] = ((uint64_t)hi[2 * k] << 32) | hi[2 * k + 1];
    sha512_compress(st, w);
}

template <int MODE>
__global__ void __launch_bounds__(64)
k_pdf_r6(dprf_enum e, dprf_pdf_params p, const dprf_aes_tables *T, dprf_results *R, uint32_t cap,
         uint32_t stop_on_first, uint32_t pat_words) {
    extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
    aes_lds &L = *(aes_lds *)smem;                                  /* 2.5 KB */
    uint8_t *cs = (uint8_t *)(smem + sizeof(aes_lds) / 4);          /* 256 B */
    uint32_t *flag = smem + sizeof(aes_lds) / 4 + 64;
    uint8_t *pat = (uint8_t *)(smem + sizeof(aes_lds) / 4 + 64 + 4); /* pat_words * 256 B */
    const uint32_t tid = threadIdx.x;
    for (uint32_t k = tid; k < 64; k += 64) ((uint32_t *)cs)[k] = ((const uint32_t *)e.charset)[k];
    for (uint32_t k = tid; k < 256; k += 64) { L.te[k] = T->te0[k]; L.td[k] = T->td0[k]; }
    for (uint32_t k = tid; k < 64; k += 64) { L.sb[k] = ((const uint32_t *)T->sbox)[k]; L.isb[k] = ((const uint32_t *)T->inv_sbox)[k]; }
    if (tid == 0) *flag = stop_on_first ? __hip_atomic_load(&R->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
    __syncthreads();
    if (*flag) return;

    const uint32_t g0 = blockIdx.x * blockDim.x + tid;
    const bool valid = g0 < e.count;
    const uint32_t g = valid ? g0 : e.count - 1;
    cand6 c;
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) c.w[j] = 0;
    if (MODE == 0) {
        uint32_t rem = g, carry = 0;
#pragma unroll
        for (int pp = DPRF_MAX_RANGE_LEN - 1; pp >= 0; --pp) {
            if ((uint32_t)pp < e.pwlen) {
                uint32_t q = e.cslen == 1 ? rem : fastdiv6(rem, e.div_m, e.div_s);
                uint32_t r = rem - q * e.cslen;
                uint32_t d = (uint32_t)e.sdig[pp] + r + carry;
                carry = d >= e.cslen ? 1u : 0u;
                d -= carry ? e.cslen : 0u;
                rem = q;
                c.w[pp >> 2] |= (uint32_t)cs[d] << (8 * (pp & 3));
            }
        }
        c.len = e.pwlen;
    } else {
        const uint64_t slot = e.start + g;
        const uint4 *s = (const uint4 *)(e.slots + slot * DPRF_SLOT_WORDS);
#pragma unroll
        for (int q = 0; q < DPRF_SLOT_WORDS / 4; q++) {
            uint4 v = s[q];
            c.w[4 * q] = v.x; c.w[4 * q + 1] = v.y; c.w[4 * q + 2] = v.z; c.w[4 * q + 3] = v.w;
        }
        c.len = e.lens[slot];
    }
    const uint32_t len = c.len;
    const uint32_t lanebase = tid << 2;

    /* K = SHA256(pw || salt8) (:240-245): LE message with the salt at byte offset len */
    uint32_t K[16];
    {
        uint32_t m[32];
#pragma unroll
        for (int j = 0; j < 32; j++) m[j] = j < DPRF_SLOT_WORDS ? (c.w[j] & le_keep_mask(j, len)) : 0u;
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
    }
    /* the password bytes at the head of the pattern never change: word-aligned, written once (bytes
     * past len are overwritten by K below) */
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) *(uint32_t *)(pat + (((uint32_t)j << 8) | lanebase)) = c.w[j];

    uint32_t bs = 32, last = 0, done = 0;
    for (uint32_t i = 0; ; i++) {
        if (!__any(!done)) break;
        const bool act = !done;
        const uint32_t Lp = len + bs;
        if (act) {
            /* pattern = pw || K[0:bs] || pw || K[0:bs] (two periods, so a 16-byte read never wraps) */
#pragma unroll
            for (int k = 0; k < 64; k++) {
                if ((uint32_t)k < bs) {
                    const uint32_t b = (K[k >> 2] >> (24 - 8 * (k & 3))) & 0xffu;
                    pat[pat_addr(len + k, lanebase)] = (uint8_t)b;
                    pat[pat_addr(Lp + len + k, lanebase)] = (uint8_t)b;
                }
            }
            for (uint32_t k = 0; k < len; k++) pat[pat_addr(Lp + k, lanebase)] = pat[pat_addr(k, lanebase)];
        }
        /* AES-128 key K[0:16], iv K[16:32] (:259-261) */
        uint32_t rk[44];
        aes128_expand(L, K, rk);
        uint32_t prev[4] = {K[4], K[5], K[6], K[7]};
        uint32_t st256[8];
        uint64_t st512[8];
        uint32_t half[16];
        uint32_t hsel = 0;      /* 0: SHA-256, 1: SHA-384, 2: SHA-512 */
        uint32_t o = 0;         /* byte offset of the next plaintext block within the period */
        uint32_t elast = 0;
        for (uint32_t u = 0; u < Lp; u++) {          /* 64-byte units; per-lane trip count */
            if (!act) break;
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t wi = o >> 2, sh = o & 3u;
                const uint32_t sel = 0x00010203u + sh * 0x01010101u;
                uint32_t lw[5];
#pragma unroll
                for (int k = 0; k < 5; k++) lw[k] = *(const uint32_t *)(pat + (((wi + k) << 8) | lanebase));
                uint32_t x[4], y[4];
#pragma unroll
                for (int k = 0; k < 4; k++) x[k] = perm(lw[k + 1], lw[k], sel) ^ prev[k];
                aes_encrypt<10>(L, rk, x, y);
#pragma unroll
                for (int k = 0; k < 4; k++) { prev[k] = y[k]; w[4 * q + k] = y[k]; }
                o += 16u;
                o = o >= Lp ? o - Lp : o;
                if (u == 0 && q == 0) {
                    /* Step 4: SHA-2 size for this round from sum(E[0:16]) mod 3 (:264-268) */
                    uint32_t sum = __builtin_amdgcn_sad_u8(y[0], 0u, 0u);
                    sum = __builtin_amdgcn_sad_u8(y[1], 0u, sum);
                    sum = __builtin_amdgcn_sad_u8(y[2], 0u, sum);
                    sum = __builtin_amdgcn_sad_u8(y[3], 0u, sum);
                    hsel = sum % 3u;
                    if (hsel == 0) sha256_iv(st256);
                    else sha512_iv(st512, hsel == 1);
                }
            }
            if (hsel == 0) {
                sha256_compress(st256, w);
            } else if (u & 1u) {
                sha512_compress_w32(st512, half, w);
            } else {
#pragma unroll
                for (int k = 0; k < 16; k++) half[k] = w[k];
            }
        }
        if (act) {
            elast = prev[3] & 0xffu;
            const uint32_t total = 64u * Lp, bits = total * 8u;
            if (hsel == 0) {
                uint32_t w[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
                sha256_compress(st256, w);
#pragma unroll
                for (int k = 0; k < 8; k++) K[k] = st256[k];
#pragma unroll
                for (int k = 8; k < 16; k++) K[k] = 0u;
            } else {
                uint32_t w[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
                if (Lp & 1u) {
                    sha512_compress_w32(st512, half, w);
                } else {
                    uint32_t z[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
                    uint32_t w2[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, bits};
                    sha512_compress_w32(st512, z, w2);
                }
#pragma unroll
                for (int k = 0; k < 8; k++) { K[2 * k] = (uint32_t)(st512[k] >> 32); K[2 * k + 1] = (uint32_t)st512[k]; }
                if (hsel == 1) {
#pragma unroll
                    for (int k = 12; k < 16; k++) K[k] = 0u;
                }
            }
            bs = 32u + 16u * hsel;
            last = elast;
            /* loop condition of :247, evaluated with i+1 */
            if (i + 1u >= 64u && i + 1u >= last + 32u) done = 1;
        }
    }
    bool ok = true;
#pragma unroll
    for (int k = 0; k < 8; k++) ok = ok && K[k] == p.u[k];
    if (valid && ok) {
        uint32_t slot = atomicAdd(&R->nhits, 1u);
        if (slot < cap) R->hits[slot] = e.start + g;
        atomicMin(&R->first, (unsigned long long)(e.start + g));
        if (stop_on_first) atomicExch(&R->stop, 1u);
    }
    if (tid == 0) {
        uint32_t base = blockIdx.x * blockDim.x;
        uint32_t n = e.count - base < blockDim.x ? e.count - base : blockDim.x;
        atomicAdd(&R->evaluated, (unsigned long long)n);
    }
}

hipError_t launch_pdf_r6(const dprf_enum &e, const dprf_pdf_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s) {
    const uint32_t lmax = e.mode == 0 ? e.pwlen : 4u * DPRF_SLOT_WORDS;
    const uint32_t pat_words = (2u * (lmax + 64u) + 3u) / 4u + 1u;
    const size_t shm = sizeof(aes_lds) + 256 + 16 + (size_t)pat_words * 256u;
    dim3 grid((e.count + 63) / 64);
    if (e.mode == 0) hipLaunchKernelGGL(k_pdf_r6<0>, grid, dim3(64), shm, s, e, p, T, R, cap, stop, pat_words);
    else hipLaunchKernelGGL(k_pdf_r6<1>, grid, dim3(64), shm, s, e, p, T, R, cap, stop, pat_words);
    return hipGetLastError();
}

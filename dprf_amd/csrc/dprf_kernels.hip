/* dprf_kernels.hip -- gfx950 verification kernels, one candidate per lane.
 *
 * Each kernel restates one reference verify() for a batch of candidates:
 *   k_office_kdf + k_office_check   msoffcrypto_password_verifier.c:56-191  (SHA-1 x50,002; AES-128-ECB check)
 *   k_odt_kdf + k_odt_check         odt_password_verifier.c:51-126  (SHA-256, PBKDF2-HMAC-SHA1 x1024; AES-256-CBC)
 *   k_pdf_r24  pdf_password_verifier.c:134-191         (MD5 [x50] + RC4 [x20], S-box in LDS)
 *   k_pdf_r5   pdf_password_verifier.c:194-221         (one SHA-256)
 *   k_pdf_r6   pdf_password_verifier.c:226-291         (dprf_kernels_r6.hip)
 * Candidates come either from on-device enumeration of a keyspace index (range mode, the
 * brute_force.py -pr path) or from a packed slot buffer (list mode, the client payload path).
 * A hit appends its index to a device buffer (atomic), lowers `first` (atomicMin) and, when asked,
 * raises a stop flag that later launches of the same call observe and skip.
 */
#include "dev_crypto.h"
#include "dprf_params.h"
#include "dprf_launch.h"
#include "dprf_hits.h"
#include "rc4_dev.h"

/* ------------------------------------------------------------------ candidate source */
struct cand {
    uint32_t w[DPRF_SLOT_WORDS];   /* LE-packed bytes (UTF-16LE code units for Office) */
    uint32_t len;                  /* bytes */
};

DEVI uint32_t fastdiv(uint32_t n, uint32_t m, uint32_t s) {
    uint32_t t = __umulhi(n, m);
    return (t + ((n - t) >> 1)) >> s;
}

/* Keyspace index start+g -> candidate, itertools.product order (brute_force.py:205): the digit at
 * position pwlen-1 varies fastest.  UTF16: emit UTF-16LE code units (Office; ASCII charset only). */
template <bool UTF16>
DEVI void range_candidate(const dprf_enum &e, const uint8_t *cs, uint32_t g, cand &c) {
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) c.w[j] = 0;
    uint32_t rem = g, carry = 0;
#pragma unroll
    for (int p = DPRF_MAX_RANGE_LEN - 1; p >= 0; --p) {
        if ((uint32_t)p < e.pwlen) {
            uint32_t q = e.cslen == 1 ? rem : fastdiv(rem, e.div_m, e.div_s);
            uint32_t r = rem - q * e.cslen;
            uint32_t d = (uint32_t)e.sdig[p] + r + carry;
            carry = d >= e.cslen ? 1u : 0u;
            d -= carry ? e.cslen : 0u;
            rem = q;
            uint32_t ch = cs[d];
            if (UTF16) c.w[p >> 1] |= ch << (16 * (p & 1));
            else c.w[p >> 2] |= ch << (8 * (p & 3));
        }
    }
    c.len = UTF16 ? 2 * e.pwlen : e.pwlen;
}

DEVI void list_candidate(const dprf_enum &e, uint32_t g, cand &c) {
    const uint64_t slot = e.start + g;
    const uint4 *s = (const uint4 *)(e.slots + slot * DPRF_SLOT_WORDS);
#pragma unroll
    for (int q = 0; q < DPRF_SLOT_WORDS / 4; q++) {
        uint4 v = s[q];
        c.w[4 * q + 0] = v.x; c.w[4 * q + 1] = v.y; c.w[4 * q + 2] = v.z; c.w[4 * q + 3] = v.w;
    }
    c.len = e.lens[slot];
}

template <int MODE, bool UTF16>
DEVI void get_candidate(const dprf_enum &e, const uint8_t *cs, uint32_t g, cand &c) {
    if (MODE == 0) range_candidate<UTF16>(e, cs, g, c);
    else list_candidate(e, g, c);
}

/* ------------------------------------------------------------------ block prologue / epilogue */
/* Stage the charset (and optionally the AES tables) into LDS and decide once per block whether it runs.
 * With stop_on_first a block is skipped only when its LOWEST candidate index lies above the lowest hit
 * known so far (R->first, and across devices the call's, dprf_hits.h): every index below the final `first` is then verified whatever order the
 * workgroups are dispatched in, so the reported hit is the lowest of the call unconditionally (a boolean
 * stop flag would let a late-dispatched lower block skip itself).  `per` = candidates per thread.
 * COUNT: this kernel's skipped blocks are counted in R->skipped (the verifying kernel of a format; the
 * KDF kernels of Office/ODF skip exactly the blocks their check kernel skips and do not count). */
template <bool AES, bool COUNT = true, bool STAGE_CS = true>
DEVI bool block_prologue(const dprf_enum &e, const dprf_aes_tables *T, dprf_results *R, uint32_t stop_on_first,
                         uint8_t *cs, aes_lds *L, uint32_t *flag, uint32_t per = 1) {
    const uint32_t tid = threadIdx.x;
    if (STAGE_CS)
        for (uint32_t k = tid; k < 64; k += blockDim.x) ((uint32_t *)cs)[k] = ((const uint32_t *)e.charset)[k];
    if (AES) {
        for (uint32_t k = tid; k < 256; k += blockDim.x) { L->te[k] = T->te0[k]; L->td[k] = T->td0[k]; }
        for (uint32_t k = tid; k < 64; k += blockDim.x) {
            L->sb[k] = ((const uint32_t *)T->sbox)[k];
            L->isb[k] = ((const uint32_t *)T->inv_sbox)[k];
        }
    }
    if (tid == 0) {
        uint32_t skip = 0u;
        if (stop_on_first) {
            const uint32_t off = blockIdx.x * blockDim.x * per;
            skip = e.start + off > lowest_known(e, R) ? 1u : 0u;
            if (skip && COUNT) {
                const uint32_t n = e.count - off < blockDim.x * per ? e.count - off : blockDim.x * per;
                atomicAdd(&R->skipped, (unsigned long long)n);
            }
        }
        *flag = skip;
    }
    __syncthreads();
    return *flag == 0;
}


/* BE message words of `len` candidate bytes (LE-packed) placed after `pre` bytes already in m[],
 * pre a multiple of 4 and <= 16, with the 0x80 terminator.  Static indices only.  A candidate that fills its whole
 * 64-byte slot (Office: 32 UTF-16 units; ODF: 64 bytes) has its terminator in the word after the slot (round 5: until
 * then it was dropped, and such a password was never found). */
template <int PREW>
DEVI void be_append(uint32_t m[32], const cand &c) {
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++)
        m[PREW + j] = bswap32((c.w[j] & le_keep_mask(j, c.len)) | le_pad80(j, c.len));
#pragma unroll
    for (int j = PREW + DPRF_SLOT_WORDS; j < 32; j++) m[j] = 0;
    m[PREW + DPRF_SLOT_WORDS] = c.len == 4u * DPRF_SLOT_WORDS ? 0x80000000u : 0u;
}

/* SHA-1 / SHA-256 of a <= 119-byte message held in m[32] (BE, already terminated with 0x80):
 * one or two blocks, chosen per lane. */
DEVI void sha1_msg2(uint32_t m[32], uint32_t total, uint32_t out[5]) {
    const uint32_t bits = total * 8u;
    const bool two = total > 55u;
    uint32_t b0[16], b1[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { b0[j] = m[j]; b1[j] = m[16 + j]; }
    if (!two) b0[15] = bits;
    b1[15] = bits;
    sha1_iv(out);
    sha1_compress(out, b0);
    if (two) sha1_compress(out, b1);
}
DEVI void sha256_msg2(uint32_t m[32], uint32_t total, uint32_t out[8]) {
    const uint32_t bits = total * 8u;
    const bool two = total > 55u;
    uint32_t b0[16], b1[16];
#pragma unroll
    for (int j = 0; j < 16; j++) { b0[j] = m[j]; b1[j] = m[16 + j]; }
    if (!two) b0[15] = bits;
    b1[15] = bits;
    sha256_iv(out);
    sha256_compress(out, b0);
    if (two) sha256_compress(out, b1);
}

/* The file is compiled three times (Makefile): the Office kernels (DPRF_PART_OFFICE), the ODF kernels
 * (DPRF_PART_ODT) and the PDF R2-R5 kernels (DPRF_PART_PDF), each object with the LLVM machine-scheduler
 * strategy that measured fastest for it AND leaves its kernels without scratch (resource_gate.py). */
#if !defined(DPRF_PART_OFFICE) && !defined(DPRF_PART_ODT) && !defined(DPRF_PART_PDF) && !defined(DPRF_PART_LONG)
#define DPRF_PART_OFFICE
#define DPRF_PART_ODT
#define DPRF_PART_PDF
#define DPRF_PART_LONG
#endif

#ifdef DPRF_PART_LONG
/* ================================================================== long candidates (round 4) */
/* Candidates longer than the 64-byte list slot: the reference hashes any strlen(password) -- ODF's start key
 * (odt...c:78-79), Office's H0 over salt || UTF-16LE (msoffcrypto...c:94-101, iconv of any length :275-336), PDF R5
 * after truncation at 127 (pdf...c:197-206) and R6's K0 over the whole password (:240-245, <= 176 bytes, :228).  This
 * kernel computes that first message's hash for one record per lane, streaming the record from the blob in 64-byte
 * blocks (a lane loops over its own block count; records are rare, so the divergence costs nothing that matters);
 * the format's usual kernels then run from the hash in `keys` (Office / ODF KDF, R6), or it compares directly (R5).
 * Records sit 16-byte aligned in the blob, zero past their length; message words are built with static indices only. */
DEVI uint32_t long_msg_word(const uint32_t *rec, uint32_t len, uint32_t dw, const uint32_t sw[3], uint32_t ns) {
    /* LE word dw of record || suffix bytes || 0x80: the suffix words sw[0..ns) (ns - 1 suffix words + the 0x80 word)
     * land at byte offset len */
    uint32_t v = 4u * dw < len ? rec[dw] & le_keep_mask(0, len - 4u * dw) : 0u;
    const uint32_t q = len >> 2, r = (len & 3u) * 8u;
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
        if (k >= ns) break;
        if (dw == q + k) v |= sw[k] << r;
        if (r && dw == q + k + 1u) v |= sw[k] >> (32u - r);
    }
    return v;
}
__global__ void __launch_bounds__(256)
k_long_prehash(dprf_enum e, dprf_long_params lp, dprf_results *R, uint32_t cap, uint32_t stop_on_first) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= e.count) return;
    const uint64_t rec = e.start + g;
    const uint32_t *d = e.slots + e.loff[rec];
    const uint32_t len = e.llen[rec];
    const bool sha1 = lp.alg == DPRF_LONG_SHA1_SALT16;
    const uint32_t prew = sha1 ? 4u : 0u;                                /* message words before the record */
    const bool salt = lp.alg == DPRF_LONG_SHA256_SALT8 || lp.alg == DPRF_LONG_R5;
    const uint32_t sw[3] = {salt ? lp.suffix[0] : 0x80u, salt ? lp.suffix[1] : 0u, 0x80u};
    const uint32_t ns = salt ? 3u : 1u;
    const uint32_t total = 4u * prew + len + (salt ? 8u : 0u);           /* message bytes */
    const uint32_t nb = (total + 9u + 63u) >> 6;                        /* blocks incl. 0x80 and the bit length */
    uint32_t h[8];
    if (sha1) { sha1_iv(h); h[5] = h[6] = h[7] = 0u; }
    else sha256_iv(h);
    for (uint32_t b = 0; b < nb; b++) {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t t = 16u * b + (uint32_t)j;
            w[j] = t < prew ? lp.prefix[j & 3] : bswap32(long_msg_word(d, len, t - prew, sw, ns));
        }
        if (b + 1u == nb) { w[14] = 0u; w[15] = total * 8u; }
        if (sha1) sha1_compress(h, w);
        else sha256_compress(h, w);
    }
    if (lp.alg == DPRF_LONG_R5) {
        bool ok = true;
#pragma unroll
        for (int k = 0; k < 8; k++) ok = ok && h[k] == lp.target[k];
        if (ok) report_hit(e, R, rec, cap, stop_on_first);
        return;
    }
#pragma unroll
    for (int k = 0; k < 8; k++)
        if (k < 5 || !sha1) e.keys[(size_t)k * e.count + g] = h[k];
}

/* ================================================================== symbol windows (round 6) */
/* Range mode over a charset whose symbols take several bytes (a --charset with non-ASCII characters: one symbol per
 * character, its UTF-8 -- for Office its UTF-16LE -- bytes): index g of the chunk -> the candidate's bytes in a list
 * slot, in itertools.product order over the symbols (brute_force.py:205), for the list-mode kernels to verify.  The
 * digits come as in range_candidate (the chunk start's digits from the host, g added with carries); the bytes are
 * assembled in the thread's column of an LDS tile and the block's slots leave it as consecutive 16-byte pieces.
 * Bytes at or past `trunc` (PDF R2-R4 hash 32, pdf...c:137) and past the slot are never written: the slot stays zero
 * there, as dprf_verify_list packs a truncated candidate. */
__global__ void __launch_bounds__(256)
k_spell_symbols(dprf_enum e, const uint32_t *symtab, uint32_t trunc, uint32_t *slots, uint8_t *lens) {
    /* the block's 256 slots as [word][slot] with a row stride of 258 words: the byte stores of one word index and the
     * 16-byte read-outs below both spread over the banks */
    constexpr uint32_t ST = 258;
    __shared__ uint32_t sym[256], syl[256];
    __shared__ uint32_t tile[DPRF_SLOT_WORDS * ST];
    const uint32_t tid = threadIdx.x;
    sym[tid] = symtab[tid];
    syl[tid] = symtab[256 + tid];
#pragma unroll
    for (int j = 0; j < DPRF_SLOT_WORDS; j++) tile[j * ST + tid] = 0u;
    __syncthreads();
    const uint32_t g = blockIdx.x * 256u + tid;
    const uint32_t n = e.pwlen < DPRF_MAX_RANGE_LEN ? e.pwlen : DPRF_MAX_RANGE_LEN;
    const uint32_t lim = trunc < 4u * DPRF_SLOT_WORDS ? trunc : 4u * DPRF_SLOT_WORDS;
    if (g < e.count) {
        /* the digits twice, last position first (as range_candidate): once for the length, once to store each
         * symbol's bytes right to left from it -- no digit array */
        uint32_t total = 0;
        for (int pass = 0; pass < 2; pass++) {
            uint32_t rem = g, carry = 0, pos = total;
            for (int p = (int)n - 1; p >= 0; --p) {
                const uint32_t q = e.cslen == 1 ? rem : fastdiv(rem, e.div_m, e.div_s);
                uint32_t d = (uint32_t)e.sdig[p] + (rem - q * e.cslen) + carry;
                carry = d >= e.cslen ? 1u : 0u;
                d -= carry ? e.cslen : 0u;
                rem = q;
                const uint32_t k = syl[d];
                if (pass == 0) {
                    total += k;
                } else {
                    pos -= k;
                    const uint32_t w = sym[d];
                    uint8_t *tb = (uint8_t *)tile;
                    for (uint32_t j = 0; j < k; j++)
                        if (pos + j < lim) tb[4u * (((pos + j) >> 2) * ST + tid) + ((pos + j) & 3u)] = (uint8_t)(w >> (8u * j));
                }
            }
        }
        lens[g] = (uint8_t)(total < lim ? total : lim);
    }
    __syncthreads();
    /* read-out: 16-byte piece u = 256 q + tid of the block's 16 KB of slots (slot u / 4, words 4 (u % 4) ..), so every
     * store instruction of the block writes 4 KB of consecutive memory */
    const uint32_t base = blockIdx.x * 256u;
    uint4 *out = (uint4 *)(slots + (size_t)base * DPRF_SLOT_WORDS);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const uint32_t u = 256u * q + tid, sl = u >> 2, w0 = 4u * (u & 3u);
        if (base + sl < e.count)
            out[u] = make_uint4(tile[w0 * ST + sl], tile[(w0 + 1) * ST + sl], tile[(w0 + 2) * ST + sl],
                                tile[(w0 + 3) * ST + sl]);
    }
}
#endif /* DPRF_PART_LONG */

#ifdef DPRF_PART_OFFICE
/* ================================================================== Office (ECMA-376 Standard) */
/* Two launches per batch.  k_office_kdf runs the 50,002 dependent SHA-1s at 8 waves/SIMD (<= 64 VGPRs)
 * and leaves the AES-128 key X1[0:16] of every candidate in HBM ([word][candidate], coalesced);
 * k_office_check does the AES-128 verifier check with its own register budget.  The hand-off costs
 * 32 bytes per candidate against ~3e7 issue slots of hashing. */
template <int MODE>
__global__ void __launch_bounds__(256, 8)
k_office_kdf(dprf_enum e, dprf_office_params p, dprf_results *R, uint32_t stop_on_first, uint32_t *keys) {
    __shared__ uint8_t cs[256];
    __shared__ uint32_t flag;
    if (!block_prologue<false, false>(e, nullptr, R, stop_on_first, cs, nullptr, &flag)) return;
    const uint32_t g0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (g0 >= e.count) return;
    const uint32_t g = g0;
    uint32_t h[5];
    if constexpr (MODE == 2) {
        /* long list: H0 from k_long_prehash (same place this kernel leaves X1: the lane's own column) */
#pragma unroll
        for (int k = 0; k < 5; k++) h[k] = keys[(size_t)k * e.count + g];
    } else {
        cand c;
        get_candidate<MODE, true>(e, cs, g, c);
        /* H0 = SHA1(salt[0:16] || UTF16LE(pw)) (msoffcrypto...c:94-101) */
        uint32_t m[32];
        m[0] = p.salt[0]; m[1] = p.salt[1]; m[2] = p.salt[2]; m[3] = p.salt[3];
        be_append<4>(m, c);
        sha1_msg2(m, 16u + c.len, h);
    }

    /* 50,000 x H = SHA1(LE32(i) || H) (:105-113): W0 = bswap(i) is wave-uniform */
    for (uint32_t i = 0; i < 50000u; i++) {
        uint32_t w[16] = {bswap32(i), h[0], h[1], h[2], h[3], h[4], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 192u};
        uint32_t s[5];
        sha1_iv(s);
        sha1_compress(s, w);
        h[0] = s[0]; h[1] = s[1]; h[2] = s[2]; h[3] = s[3]; h[4] = s[4];
    }
    /* H = SHA1(H || 00000000) (:115-118) */
    {
        uint32_t w[16] = {h[0], h[1], h[2], h[3], h[4], 0u, 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 192u};
        sha1_iv(h);
        sha1_compress(h, w);
    }
    /* X1 = SHA1((0x36 x 64) ^ H), key = X1[0:16] (:128-153) */
    uint32_t x1[5];
    {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = 0x36363636u ^ (j < 5 ? h[j] : 0u);
        sha1_iv(x1);
        sha1_compress(x1, w);
        uint32_t w2[16] = {0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 512u};
        sha1_compress(x1, w2);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) keys[(size_t)k * e.count + g] = x1[k];
}

__global__ void __launch_bounds__(256)
k_office_check(dprf_enum e, dprf_office_params p, const dprf_aes_tables *T, dprf_results *R, uint32_t cap,
               uint32_t stop_on_first, const uint32_t *keys) {
    __shared__ uint8_t cs[256];
    __shared__ aes_lds L;
    __shared__ uint32_t flag;
    if (!block_prologue<true>(e, T, R, stop_on_first, cs, &L, &flag)) return;
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = g < e.count;
    uint32_t key[4];
#pragma unroll
    for (int k = 0; k < 4; k++) key[k] = valid ? keys[(size_t)k * e.count + g] : 0u;
    /* AES-128-ECB decrypt of verifier and verifier hash, always AES-128 (:159-172, :207) */
    uint32_t rk[44], dk[44];
    aes128_expand(L, key, rk);
    aes_dec_schedule<10>(L, rk, dk);
    uint32_t dv[4], dh0[4], dh1[4];
    aes_decrypt<10>(L, dk, p.ev, dv);
    aes_decrypt<10>(L, dk, p.evh, dh0);
    aes_decrypt<10>(L, dk, p.evh + 4, dh1);
    /* decryptedVerifierHash[hash_size] == 0 (:168), hash_size uniform in [0,32) */
    const uint32_t hs = p.hash_size;
    const uint32_t wi = (hs & 15u) >> 2, sh = 24u - 8u * (hs & 3u);
    uint32_t word;
    if (hs < 16u) word = wi == 0 ? dh0[0] : wi == 1 ? dh0[1] : wi == 2 ? dh0[2] : dh0[3];
    else word = wi == 0 ? dh1[0] : wi == 1 ? dh1[1] : wi == 2 ? dh1[2] : dh1[3];
    bool ok = ((word >> sh) & 0xffu) == 0u;
    /* SHA1(verifier) == dec_evh[0:20] (:175-188) */
    uint32_t vh[5];
    {
        uint32_t w[16] = {dv[0], dv[1], dv[2], dv[3], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 128u};
        sha1_iv(vh);
        sha1_compress(vh, w);
    }
    ok = ok && vh[0] == dh0[0] && vh[1] == dh0[1] && vh[2] == dh0[2] && vh[3] == dh0[3] && vh[4] == dh1[0];
    if (valid && ok) report_hit(e, R, e.start + g, cap, stop_on_first);
}

#endif /* DPRF_PART_OFFICE */

#ifdef DPRF_PART_ODT
/* ================================================================== ODF 1.2 (AES-256-CBC, PBKDF2-HMAC-SHA1) */
/* Two launches per batch, as for Office: k_odt_kdf (SHA-256 start key + PBKDF2, 8 waves/SIMD) leaves the
 * 32-byte AES-256 key of every candidate in HBM; k_odt_check decrypts and verifies. */
#ifndef ODT_KDF_WAVES
#define ODT_KDF_WAVES 6             /* waves per SIMD: 8 / 6 / 4 measured the same (round 2); 6 leaves room for sha1_pre */
#endif
template <int MODE>
__global__ void __launch_bounds__(256, ODT_KDF_WAVES)
k_odt_kdf(dprf_enum e, dprf_odt_params p, dprf_results *R, uint32_t stop_on_first, uint32_t *keys) {
    __shared__ uint8_t cs[256];
    __shared__ uint32_t flag;
    if (!block_prologue<false, false>(e, nullptr, R, stop_on_first, cs, nullptr, &flag)) return;
    const uint32_t g0 = blockIdx.x * blockDim.x + threadIdx.x;
    if (g0 >= e.count) return;
    const uint32_t g = g0;
    /* start key = SHA256(password) (odt...c:78-79) */
    uint32_t sk[8];
    if constexpr (MODE == 2) {
        /* long list: from k_long_prehash, in the lane's own key column */
#pragma unroll
        for (int k = 0; k < 8; k++) sk[k] = keys[(size_t)k * e.count + g];
    } else {
        cand c;
        get_candidate<MODE, false>(e, cs, g, c);
        uint32_t m[32];
        be_append<0>(m, c);
        sha256_msg2(m, c.len, sk);
    }
    /* PBKDF2-HMAC-SHA1(sk, salt, 1024, 32) (:85): ipad/opad midstates once per candidate */
    uint32_t ist[5], ost[5];
    {
        uint32_t w[16];
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = 0x36363636u ^ (j < 8 ? sk[j] : 0u);
        sha1_iv(ist); sha1_compress(ist, w);
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = 0x5c5c5c5cu ^ (j < 8 ? sk[j] : 0u);
        sha1_iv(ost); sha1_compress(ost, w);
    }
    /* the midstates' message-independent parts of rounds 0-4, once per candidate (dev_crypto.h sha1_pre) */
    const sha1_pre_t ipre = sha1_pre(ist), opre = sha1_pre(ost);
#pragma unroll
    for (int blkno = 1; blkno <= 2; blkno++) {
        uint32_t u[5], t[5];
        {
            uint32_t w[16] = {p.salt[0], p.salt[1], p.salt[2], p.salt[3], (uint32_t)blkno, 0x80000000u,
                              0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 20u) * 8u};
            uint32_t s[5];
            sha1_compress_pre(ist, ipre, w, s);
            uint32_t w2[16] = {s[0], s[1], s[2], s[3], s[4], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 20u) * 8u};
            sha1_compress_pre(ost, opre, w2, u);
        }
        t[0] = u[0]; t[1] = u[1]; t[2] = u[2]; t[3] = u[3]; t[4] = u[4];
        for (int it = 1; it < 1024; it++) {
            uint32_t w[16] = {u[0], u[1], u[2], u[3], u[4], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 20u) * 8u};
            uint32_t s[5];
            sha1_compress_pre(ist, ipre, w, s);
            uint32_t w2[16] = {s[0], s[1], s[2], s[3], s[4], 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, (64u + 20u) * 8u};
            sha1_compress_pre(ost, opre, w2, u);
            t[0] ^= u[0]; t[1] ^= u[1]; t[2] ^= u[2]; t[3] ^= u[3]; t[4] ^= u[4];
        }
        /* each block's key words go out as soon as they are known (block 1's five need not stay live through
         * block 2) */
        if (blkno == 1) {
#pragma unroll
            for (int k = 0; k < 5; k++) keys[(size_t)k * e.count + g] = t[k];
        } else {
#pragma unroll
            for (int k = 0; k < 3; k++) keys[(size_t)(5 + k) * e.count + g] = t[k];
        }
    }
}

/* The 64 AES-256 block decryptions per candidate read Td0 14,336 times.  A single 1 KiB Td0 puts
 * random indices of 32 lanes on 32 banks (~3.5-way conflicts: 65 % of this kernel's cycles were bank
 * conflicts, profiles/prof_odt_r01.json).  The tables follow R6's split-table scheme (dprf_kernels_r6.hip
 * aes128_encrypt_split; the replicated single table of rounds 1-2, 12 v_alignbit per round, is in HISTORY.md) for
 * the inverse cipher: four tables Td_t = ror(Td0, 8t) x 16 copies fill the 256-byte rows, lane group A (bit 4 of the lane clear) reads
 * Td_t and group B Td_t+1 in every lookup (32 different banks per 32-lane half), B keeps its state rotated -- after
 * inner round r its register j holds ror(s_(j + rho_r), 8 eps_r) with (rho, eps) -> (rho - eps, eps + 1) for the
 * inverse cipher's column order -- and its round keys are permuted to match; no rotates are left.  Si sits in one
 * more row (address 0x10000 + x, one v_perm; the last round's 16 byte reads share its banks).
 * tests/test_odt_split_model.py restates it against FIPS-197. */
#define ODT_TD_ROW 256
__shared__ __attribute__((aligned(16))) uint32_t odt_td[(256 + 1) * ODT_TD_ROW / 4];

/* B's representation (rho, eps) after inner round r = 0..13 of the inverse cipher */
__device__ constexpr int ODT_RHO[14] = {0, 0, 3, 1, 2, 2, 1, 3, 0, 0, 3, 1, 2, 2};
__device__ constexpr int ODT_EPS[14] = {0, 1, 2, 3, 0, 1, 2, 3, 0, 1, 2, 3, 0, 1};
#define ODT_SEL(t) (0x0c0c0000u | ((4u + 3u - (t)) << 8) | (t))
/* One inner round: 16 lookups issued column by column (column j: s_j, s_j-1, s_j-2, s_j-3 for lookups t = 0..3),
 * then each column's two v_bitop3 behind the wait covering its reads (as r6_round_asm). */
DEVI void odt_round_asm(uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3, uint32_t base, uint32_t k0,
                        uint32_t k1, uint32_t k2, uint32_t k3) {
    uint32_t t[16];
#define ODL(d, s, sel) "v_perm_b32 %" #d ", %" #s ", %20, %" #sel "\n\tds_read_b32 %" #d ", %" #d "\n\t"
    asm volatile(
        ODL(4, 0, 25) ODL(5, 3, 26) ODL(6, 2, 27) ODL(7, 1, 28)
        ODL(8, 1, 25) ODL(9, 0, 26) ODL(10, 3, 27) ODL(11, 2, 28)
        ODL(12, 2, 25) ODL(13, 1, 26) ODL(14, 0, 27) ODL(15, 3, 28)
        ODL(16, 3, 25) ODL(17, 2, 26) ODL(18, 1, 27) ODL(19, 0, 28)
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
        : "v"(base), "v"(k0), "v"(k1), "v"(k2), "v"(k3), "s"(ODT_SEL(0)), "s"(ODT_SEL(1)), "s"(ODT_SEL(2)),
          "s"(ODT_SEL(3))
        : "memory");
#undef ODL
}
/* Si[byte K of v] from the row after the tables (address 0x10000 + x) */
template <int K>
DEVI uint32_t odt_si(uint32_t v) {
    const uint32_t a = __builtin_amdgcn_perm(v, 0x00010000u, 0x0c020000u | (4u + K));
    return ((const uint8_t *)odt_td)[a];
}
/* Group B's round keys in its representation (A: unchanged) -- once per key schedule */
DEVI void odt_dk_split(uint32_t dk[60], uint32_t base) {
    const bool gb = (base & 0x40u) != 0u;
    const uint32_t sk[4] = {gb ? 0x03020100u : 0x07060504u, gb ? 0x00030201u : 0x07060504u,
                            gb ? 0x01000302u : 0x07060504u, gb ? 0x02010003u : 0x07060504u};
#pragma unroll
    for (int r = 1; r <= 14; r++) {
        const int rho = r < 14 ? ODT_RHO[r] : ODT_RHO[13] - ODT_EPS[13], eps = r < 14 ? ODT_EPS[r] : ODT_EPS[13];
        if (rho == 0 && eps == 0) continue;
        const uint32_t kk[4] = {dk[4 * r], dk[4 * r + 1], dk[4 * r + 2], dk[4 * r + 3]};
#pragma unroll
        for (int j = 0; j < 4; j++) dk[4 * r + j] = perm(kk[j], kk[(j + rho) & 3], sk[eps]);
    }
}
DEVI void aes256_decrypt_split(const uint32_t *dk, const uint32_t in[4], uint32_t out[4], uint32_t base) {
    uint32_t s[4] = {in[0] ^ dk[0], in[1] ^ dk[1], in[2] ^ dk[2], in[3] ^ dk[3]};
#pragma unroll
    for (int r = 1; r < 14; r++) odt_round_asm(s[0], s[1], s[2], s[3], base, dk[4 * r], dk[4 * r + 1], dk[4 * r + 2], dk[4 * r + 3]);
    /* last round: byte p of word j <- Si[byte p of s_(j-3+p)]; B's word j then holds ror(out[j + 1], 8) */
    uint32_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; j++)
        acc[j] = ((odt_si<3>(s[j]) << 24) | (odt_si<2>(s[(j + 3) & 3]) << 16) | (odt_si<1>(s[(j + 2) & 3]) << 8) |
                  odt_si<0>(s[(j + 1) & 3])) ^ dk[56 + j];
    const uint32_t selr = (base & 0x40u) ? 0x02010003u : 0x07060504u;
#pragma unroll
    for (int j = 0; j < 4; j++) out[j] = perm(acc[j], acc[(j + 3) & 3], selr);
}

#define ODT_CHECK_THREADS 512
__global__ void __launch_bounds__(ODT_CHECK_THREADS, 4)   /* 2 workgroups (64 KiB table each) per CU */
k_odt_check(dprf_enum e, dprf_odt_params p, const dprf_aes_tables *T, dprf_results *R, uint32_t cap,
            uint32_t stop_on_first, const uint32_t *keys) {
    __shared__ uint8_t cs[256];
    __shared__ aes_lds L;
    __shared__ uint32_t flag;
    for (uint32_t k = threadIdx.x; k < 256u * ODT_TD_ROW / 4; k += blockDim.x) {
        const uint32_t x = k >> 6, c = k & 63u;
        odt_td[k] = ror32(T->td0[x], 8u * (c >> 4));                             /* Td_(c/16), copy c % 16 */
    }
    if (threadIdx.x < 64u) {
        const uint32_t x = 4u * threadIdx.x;                                     /* the Si row at 0x10000 */
        odt_td[256u * ODT_TD_ROW / 4 + threadIdx.x] = (uint32_t)T->inv_sbox[x] | ((uint32_t)T->inv_sbox[x + 1] << 8) |
                                                     ((uint32_t)T->inv_sbox[x + 2] << 16) | ((uint32_t)T->inv_sbox[x + 3] << 24);
    }
    if (!block_prologue<true>(e, T, R, stop_on_first, cs, &L, &flag)) return;
    /* odt_round_asm uses the v_perm result as the whole LDS address: the table must sit at LDS address 0 (checked;
     * a build that ever breaks this fails loudly instead of computing wrong) */
    if ((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)odt_td != 0u) {
        if (threadIdx.x == 0) atomicOr(&R->pad_, 4u);
        return;
    }
    const uint32_t lanec = (threadIdx.x & 15u) << 2;
    /* split tables: byte t = row offset of the copy lookup t reads (A: Td_t, B: Td_t+1) */
    const uint32_t base = lanec * 0x01010101u + ((threadIdx.x & 16u) ? 0x00c08040u : 0xc0804000u);
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool valid = g < e.count;
    uint32_t key[8];
#pragma unroll
    for (int k = 0; k < 8; k++) key[k] = valid ? keys[(size_t)k * e.count + g] : 0u;
    /* AES-256-CBC decrypt, no padding (:90-92) */
    uint32_t rk[60], dk[60];
    aes256_expand(L, key, rk);
    aes_dec_schedule<14>(L, rk, dk);
    odt_dk_split(dk, base);
#define ODT_DECRYPT(dk, ct, pt) aes256_decrypt_split(dk, ct, pt, base)
    bool ok;
    if (p.enc_len == 16u) {
        /* experimental 2-byte check (:98-101) */
        uint32_t ct[4] = {p.enc[0], p.enc[1], p.enc[2], p.enc[3]}, pt[4];
        ODT_DECRYPT(dk, ct, pt);
        ok = ((pt[0] ^ p.iv[0]) >> 16) == 0x0300u;
    } else {
        /* SHA256 over the first min(len,1024) plaintext bytes == checksum (:104-123) */
        uint32_t st[8];
        sha256_iv(st);
        uint32_t prev[4] = {p.iv[0], p.iv[1], p.iv[2], p.iv[3]};
        const uint32_t n = p.hash_len, nfull = n >> 6, rem = n & 63u;
        for (uint32_t b = 0; b < nfull; b++) {
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t *cp = p.enc + (b * 4u + q) * 4u;
                uint32_t ct[4] = {cp[0], cp[1], cp[2], cp[3]}, pt[4];
                ODT_DECRYPT(dk, ct, pt);
#pragma unroll
                for (int k = 0; k < 4; k++) { w[4 * q + k] = pt[k] ^ prev[k]; prev[k] = ct[k]; }
            }
            sha256_compress(st, w);
        }
        /* final block: rem (0/16/32/48) data bytes, 0x80, bit length */
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 3; q++) {
            if ((uint32_t)q < (rem >> 4)) {
                const uint32_t *cp = p.enc + (nfull * 4u + q) * 4u;
                uint32_t ct[4] = {cp[0], cp[1], cp[2], cp[3]}, pt[4];
                ODT_DECRYPT(dk, ct, pt);
#pragma unroll
                for (int k = 0; k < 4; k++) { w[4 * q + k] = pt[k] ^ prev[k]; prev[k] = ct[k]; }
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) w[4 * q + k] = 0u;
            }
        }
#pragma unroll
        for (int k = 12; k < 16; k++) w[k] = 0u;
#pragma unroll
        for (int k = 0; k < 16; k++) if ((uint32_t)k == (rem >> 2)) w[k] = 0x80000000u;
        w[15] = n * 8u;
        sha256_compress(st, w);
        ok = true;
#pragma unroll
        for (int k = 0; k < 8; k++) ok = ok && st[k] == p.checksum[k];
    }
    if (valid && ok) report_hit(e, R, e.start + g, cap, stop_on_first);
#undef ODT_DECRYPT
}
#endif /* DPRF_PART_ODT */

#ifdef DPRF_PART_PDF
/* ================================================================== PDF R5 (one SHA-256) */
/* One SHA-256 per candidate is ~2,300 cycles of a wave: with one candidate per thread, wave launch and
 * the block prologue were a third of the kernel (2 Mi waves per 128 Mi-candidate launch).  Each thread
 * takes PER candidates: a run of PER consecutive indices in range mode when the charset has at least PER
 * characters (PER 16, or 8 for 8-15 characters: one wrap of the last digit per run at most), else -- and in
 * list mode -- PER candidates 256 apart. */
/* 1: range-mode threads take runs of consecutive candidates (below); 0: PER candidates 256 apart (A/B) */
#ifndef R5_RUNS
#define R5_RUNS 1
#endif
#ifndef R5_PER_MAX
#define R5_PER_MAX 16
#endif
/* SHA-256 of one block from the IV, compared with u[0:8], with an early exit: the last word of the digest
 * is IV7 + (e after round 60) -- that e only moves down to h in rounds 61-63 -- so a wave none of whose
 * lanes matches u[7] there (all but a 2^-32 fraction) skips rounds 61-63 and their schedule words. */
DEVI bool sha256_block_matches(uint32_t w[16], const uint32_t u[8], bool valid) {
    uint32_t a = 0x6a09e667u, b = 0xbb67ae85u, c = 0x3c6ef372u, d = 0xa54ff53au;
    uint32_t e = 0x510e527fu, f = 0x9b05688cu, g = 0x1f83d9abu, h = 0x5be0cd19u;
#pragma unroll
    for (int t = 0; t < 64; t++) {
        if (t == 61 && !__builtin_amdgcn_ballot_w64(valid && e + 0x5be0cd19u == u[7])) return false;
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = w[t & 15] + s0_256(w[(t - 15) & 15]) + w[(t - 7) & 15] + s1_256(w[(t - 2) & 15]);
            w[t & 15] = wt;
        }
        const uint32_t t1 = h + S1_256(e) + f_ch(e, f, g) + (k256(t) + wt);
        const uint32_t t2 = S0_256(a) + f_maj(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    return valid && a + 0x6a09e667u == u[0] && b + 0xbb67ae85u == u[1] && c + 0x3c6ef372u == u[2] &&
           d + 0xa54ff53au == u[3] && e + 0x510e527fu == u[4] && f + 0x9b05688cu == u[5] &&
           g + 0x1f83d9abu == u[6] && h + 0x5be0cd19u == u[7];
}
/* NW (range mode): message words 0..NW-1 carry candidate bytes (NW = ceil(pwlen / 4), one instantiation per launch
 * length); the words after them are the launch-uniform tail alone, so the compiler keeps them, K + W of their rounds
 * and the schedule terms built only from them in SGPRs (the scalar unit) instead of spending VALU slots on them */
/* minimum waves per SIMD the register allocation must allow.  Measured (round 5, profiles/ab_r5_runs_r05q.txt,
 * -pr 7 alnum, three alternating rounds): no bound (132 VGPRs, 3 waves) 32.0 G with runs of 8; 4 waves 32.86 G,
 * 5 waves 32.95 G with runs of 16 */
#ifndef R5_WAVES
#define R5_WAVES 5
#endif
template <int MODE, int NW, int PER>
__global__ void __launch_bounds__(256, R5_WAVES)
k_pdf_r5(dprf_enum e, dprf_pdf_params p, dprf_results *R, uint32_t cap, uint32_t stop_on_first) {
    static_assert(NW >= 1 && NW <= DPRF_MAX_RANGE_LEN / 4, "candidate words");
    static_assert(PER == 8 || PER == 16, "run length");
    __shared__ uint8_t cs[256];
    __shared__ uint32_t flag;
    if (!block_prologue<false>(e, nullptr, R, stop_on_first, cs, nullptr, &flag, PER)) return;
    const uint32_t base = blockIdx.x * (blockDim.x * PER);
    /* Range mode: every candidate has length pwlen <= DPRF_MAX_RANGE_LEN, so the message is one block and
     * its tail -- salt8 || 0x80 at byte pwlen, the bit length in word 15 -- is the same for the whole
     * launch: 16 uniform BE words built once (SGPRs), OR-ed onto the candidate's BE words. */
    uint32_t tail[16];
    if (MODE == 0) {
        const uint32_t len = e.pwlen, q = len >> 2, r = (len & 3u) * 8u;
        const uint32_t sw[3] = {p.u[8], p.u[9], 0x80u};
#pragma unroll
        for (int j = 0; j < 16; j++) tail[j] = 0u;
#pragma unroll
        for (int s = 0; s < 3; s++) {
            const uint32_t lo = r ? (sw[s] << r) : sw[s];
            const uint32_t hi = r ? (sw[s] >> (32u - r)) : 0u;
#pragma unroll
            for (int j = 0; j < 15; j++) {
                if ((uint32_t)j == q + s) tail[j] |= lo;
                if ((uint32_t)j == q + s + 1) tail[j] |= hi;
            }
        }
#pragma unroll
        for (int j = 0; j < 15; j++) tail[j] = bswap32(tail[j]);
        tail[15] = (len + 8u) * 8u;
    }
    if (MODE == 0 && R5_RUNS && e.cslen >= PER) {
        /* Runs (round 5): thread t takes the PER consecutive indices base + PER t + k, which differ only in the last
         * character except across one wrap of the last digit (cslen >= PER).  The candidate is spelled twice
         * per run -- at its first index (last digit d0) and at the first index past the wrap (last digit 0, prefix + 1)
         * -- as BE message words with the tail already OR-ed in and the last character cleared; each candidate then
         * costs a select per word and one charset byte instead of a full mixed-radix spelling. */
        const uint32_t g0 = base + threadIdx.x * PER;
        const uint32_t gc = g0 < e.count ? g0 : e.count - 1u;
        const uint32_t lp = e.pwlen - 1u;                             /* position of the last character */
        const uint32_t lw = lp >> 2, lsh = 24u - 8u * (lp & 3u);      /* its BE word and bit offset */
        const uint32_t q0 = e.cslen == 1 ? gc : fastdiv(gc, e.div_m, e.div_s);
        uint32_t d0 = (uint32_t)e.sdig[lp] + (gc - q0 * e.cslen);
        d0 -= d0 >= e.cslen ? e.cslen : 0u;
        uint32_t w0[NW], w1[NW];
        {
            cand c;
            range_candidate<false>(e, cs, gc, c);
#pragma unroll
            for (int j = 0; j < NW; j++) w0[j] = bswap32(c.w[j]) | tail[j];
            range_candidate<false>(e, cs, gc + (e.cslen - d0), c);
#pragma unroll
            for (int j = 0; j < NW; j++) w1[j] = bswap32(c.w[j]) | tail[j];
#pragma unroll
            for (int j = 0; j < NW; j++) {
                const uint32_t m = (uint32_t)j == lw ? ~(0xffu << lsh) : ~0u;
                w0[j] &= m; w1[j] &= m;
            }
        }
#pragma unroll 1
        for (uint32_t k = 0; k < (uint32_t)PER; k++) {
            if (base + k >= e.count) break;                             /* uniform: a wave's runs start >= base */
            const uint32_t g = g0 + k;
            const bool valid = g < e.count;
            const uint32_t d = d0 + k;
            const bool lo = d < e.cslen;
            const uint32_t ch = (uint32_t)cs[lo ? d : d - e.cslen] << lsh;
            uint32_t b[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {
                b[j] = j < NW ? (lo ? w0[j] : w1[j]) : tail[j];
                if (j < NW && (uint32_t)j == lw) b[j] |= ch;
            }
            if (sha256_block_matches(b, p.u, valid)) report_hit(e, R, e.start + g, cap, stop_on_first);
        }
        return;
    }
#pragma unroll 1
    for (uint32_t k = 0; k < (uint32_t)PER; k++) {
        const uint32_t g0 = base + k * blockDim.x + threadIdx.x;
        if (base + k * blockDim.x >= e.count) break;                 /* uniform */
        const bool valid = g0 < e.count;
        const uint32_t g = valid ? g0 : e.count - 1;
        cand c;
        get_candidate<MODE, false>(e, cs, g, c);
        if (MODE == 0) {
            /* range_candidate leaves the bytes past pwlen zero */
            uint32_t b[16];
#pragma unroll
            for (int j = 0; j < 16; j++) b[j] = (j < NW ? bswap32(c.w[j]) : 0u) | tail[j];
            if (sha256_block_matches(b, p.u, valid)) report_hit(e, R, e.start + g, cap, stop_on_first);
            continue;
        }
        if (NW < 8) {
            /* a list launch whose candidates all have at most 4 NW <= 16 bytes (launch_pdf_r5 picks NW from the
             * launch's longest): one message block, words past NW + 2 zero, and the round-61 early exit */
            uint32_t b[16];
#pragma unroll
            for (int j = 0; j < 16; j++) b[j] = j < NW ? (c.w[j] & le_keep_mask(j, c.len)) : 0u;
            const uint32_t sw[3] = {p.u[8], p.u[9], 0x80u};
            const uint32_t q = c.len >> 2, r = (c.len & 3u) * 8u;
#pragma unroll
            for (int s = 0; s < 3; s++) {
                const uint32_t lo = r ? (sw[s] << r) : sw[s];
                const uint32_t hi = r ? (sw[s] >> (32u - r)) : 0u;
#pragma unroll
                for (int j = 0; j < NW + 3; j++) {
                    if ((uint32_t)j == q + s) b[j] |= lo;
                    if ((uint32_t)j == q + s + 1) b[j] |= hi;
                }
            }
#pragma unroll
            for (int j = 0; j < NW + 3; j++) b[j] = bswap32(b[j]);
            b[15] = (c.len + 8u) * 8u;
            if (sha256_block_matches(b, p.u, valid)) report_hit(e, R, e.start + g, cap, stop_on_first);
            continue;
        }
        /* SHA256(pw[:127] || U[32:40]) == U[0:32] (pdf...c:194-221); host caps len at 127 and slots at 64 */
        uint32_t m[32];
#pragma unroll
        for (int j = 0; j < 32; j++) m[j] = j < DPRF_SLOT_WORDS ? (c.w[j] & le_keep_mask(j, c.len)) : 0u;
        /* append the 8 validation-salt bytes (LE words p.u[8], p.u[9]) at byte offset len, then 0x80 */
        const uint32_t sw[3] = {p.u[8], p.u[9], 0x80u};
        const uint32_t q = c.len >> 2, r = (c.len & 3u) * 8u;
#pragma unroll
        for (int s = 0; s < 3; s++) {
            const uint32_t lo = r ? (sw[s] << r) : sw[s];
            const uint32_t hi = r ? (sw[s] >> (32u - r)) : 0u;
#pragma unroll
            for (int j = 0; j < 32; j++) {
                if ((uint32_t)j == q + s) m[j] |= lo;
                if ((uint32_t)j == q + s + 1) m[j] |= hi;
            }
        }
#pragma unroll
        for (int j = 0; j < 32; j++) m[j] = bswap32(m[j]);
        uint32_t hh[8];
        sha256_msg2(m, c.len + 8u, hh);
        bool ok = true;
#pragma unroll
        for (int kk = 0; kk < 8; kk++) ok = ok && hh[kk] == p.u[kk];
        if (valid && ok) report_hit(e, R, e.start + g, cap, stop_on_first);
    }
}

/* ================================================================== PDF R2..R4 (MD5 + RC4) */
/* RC4 S-box layout, KSA and PRGA: rc4_dev.h */

/* RC4 key of candidate g: MD5(pw[:32] || PAD[0:32-len] || O || LE32(P) || ID [|| FFFFFFFF]) (pdf...c:136-139,
 * :352-402), then 50 x MD5(h[0:n]) for R >= 3 (:150-155).  Reads the charset and PAD from the LDS overlay. */
template <int MODE, int R, int NK>
DEVI void r24_key(const dprf_enum &e, const dprf_pdf_params &p, const uint8_t *cs, const uint32_t *padw,
                  const uint32_t padtail[8], uint32_t g, uint32_t h[4]) {
    cand c;
    get_candidate<MODE, false>(e, cs, g, c);
    const uint32_t len = c.len > 32u ? 32u : c.len;
    uint32_t pw[8];
    if (MODE == 0) {
        /* range mode: pwlen <= 32 and the bytes past it are zero; PAD at offset pwlen is launch-uniform */
#pragma unroll
        for (int j = 0; j < 8; j++) pw[j] = c.w[j] | padtail[j];
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint32_t v = c.w[j] & le_keep_mask(j, len);
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t k = 4u * j + b;
                if (k >= len) v |= (uint32_t)((const uint8_t *)padw)[k - len] << (8 * b);
            }
            pw[j] = v;
        }
    }
    {
        uint32_t m[16];
#pragma unroll
        for (int j = 0; j < 8; j++) { m[j] = pw[j]; m[8 + j] = p.tail[j]; }
        md5_iv(h);
        md5_compress(h, m);
        for (uint32_t b = 0; b < p.tail_blocks; b++) {
#pragma unroll
            for (int j = 0; j < 16; j++) m[j] = p.tail[8 + 16 * b + j];
            md5_compress(h, m);
        }
    }
    if (R >= 3) {
        for (int i = 0; i < 50; i++) {
            uint32_t m[16];
            if (NK == 16) {
                m[0] = h[0]; m[1] = h[1]; m[2] = h[2]; m[3] = h[3]; m[4] = 0x80u;
#pragma unroll
                for (int j = 5; j < 16; j++) m[j] = 0u;
                m[14] = 128u;
            } else {
                m[0] = h[0]; m[1] = (h[1] & 0xffu) | 0x8000u;
#pragma unroll
                for (int j = 2; j < 16; j++) m[j] = 0u;
                m[14] = 40u;
            }
            md5_iv(h);
            md5_compress(h, m);
        }
    }
}

/* One workgroup = one RC4 wave + one key wave, over NBAT batches of 64 candidates (round 2).
 *
 * The RC4 wave owns the workgroup's 16 KiB S-box area (one 256-byte box per lane) and only ever runs KSAs and
 * PRGAs; the key wave derives the RC4 keys (enumeration + MD5 of the padded password and document tail, and for
 * R3/R4 the 50 MD5 iterations) of batch b+1 while the RC4 wave runs batch b.  Keys are handed over through the
 * S-box area while it is free, between two barriers at each batch boundary; charset, PAD and the skip flag sit
 * in an area of their own (16,720 B per workgroup: still 9 per CU).  The RC4 wave raises its issue priority
 * (s_setprio 3), so the MD5s take only the VALU cycles the KSA chains leave free.
 * Why: when one wave did both (round 1 - mid round 2), a wave hashing its keys held its S-box without running
 * a KSA -- ~8 % of the CU's 9 KSA chains idle for R3/R4, ~15 % for R2.  Measured (tools/ab_libs.sh, MI355X):
 * R3/R4 fused 464 M, split without / with the priority 458 / 481 M; a key wave that hashes nothing (probe) 484 M,
 * so the MD5s are fully hidden; then the KSA group size re-tuned (rc4_ksa): R3/R4 513 M, R2 8.77 -> 9.79 G.
 * Batches per workgroup, R3/R4: 2 / 4 / 8 = 472 / 480 / 481 M (G = 4), 6 / 8 / 12 = 513 / 513 / 507 M (G = 2);
 * R2: 8 / 16 / 24 = 9.58 / 9.68 / 9.70 G.  Re-measured on the group-deferred KSA: R3/R4 6 / 8 / 12 batches
 * 559 / 560 / 557 M, priority 0 / 1 / 3 529 / 560 / 560 M; R2 8 / 16 / 24 batches 11.08 / 11.25 / 11.32 G,
 * priority 0 10.56 G.  Round 3 (asm KSA): 8 / 12 / 16 = 613 / 608 / 603 M; round 4, with consecutive launches on two
 * streams (the last partial generation of one launch overlaps the next): 8 / 12 / 16 = 626.2 / 628.5 / 625.2 M (three
 * alternating runs each, every run of 12 above the neighbouring 8), so 12.  R2 likewise: 16 / 24 / 36 / 48 = 12.23 /
 * 12.27 / 12.32 / 12.31 G, so 36 (profiles/ab_r2_batches_r04l.txt). */
#ifndef R34_BATCHES
#define R34_BATCHES 12
#endif
#ifndef R2_BATCHES
#define R2_BATCHES 36
#endif
#ifndef R24_PRIO
#define R24_PRIO 3
#endif
/* 1: the KSA as the generated asm block (rc4_dev.h rc4_ksa_asm); 0: the C++ rc4_ksa (A/B builds) */
#ifndef R24_KSA_ASM
#define R24_KSA_ASM 1
#endif
template <int NK>
DEVI void r24_ksa(uint8_t *S, uint32_t sbase, uint32_t lane, const uint32_t k[4]) {
    if (R24_KSA_ASM) rc4_ksa_asm<NK>(sbase, sbase + (lane << 2), k);
    else rc4_ksa<NK>(S, lane << 2, k);
}
template <int R> struct r24_batches { static constexpr uint32_t v = R == 2 ? R2_BATCHES : R34_BATCHES; };
template <int MODE, int R, int NK>
__global__ void __launch_bounds__(128, 5)   /* 18 waves per CU (9 workgroups): <= 102 VGPRs */
k_pdf_r24(dprf_enum e, dprf_pdf_params p, dprf_results *R_, uint32_t cap, uint32_t stop_on_first) {
    constexpr uint32_t NBAT = r24_batches<R>::v;
    static_assert(NBAT % 2 == 0, "block_prologue counts NBAT / 2 candidates per thread of the 128-thread block");
    __shared__ __attribute__((aligned(16))) uint8_t S[RC4_WAVE_BYTES];
    __shared__ __attribute__((aligned(16))) uint32_t aux[64 + 16 + 4];
    uint8_t *cs = (uint8_t *)aux;                         /* charset, 256 B */
    uint32_t *padw = aux + 64;                            /* PAD || PAD */
    uint32_t *flag = aux + 80;
    if (threadIdx.x < 8) { padw[threadIdx.x] = p.pad[threadIdx.x]; padw[threadIdx.x + 8] = p.pad[threadIdx.x]; }
    /* per = candidates per thread of the 128-thread block: 64 * NBAT candidates */
    if (!block_prologue<false>(e, nullptr, R_, stop_on_first, cs, nullptr, flag, NBAT / 2)) return;
    const uint32_t base = blockIdx.x * (64u * NBAT);
    const uint32_t left = e.count - base;                 /* > 0: grid = ceil(count / (64 * NBAT)) */
    const uint32_t nb = left >= 64u * NBAT ? (uint32_t)NBAT : (left + 63u) / 64u;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t *keyx = (uint32_t *)S;                       /* [4][64] words, only between the two barriers */
    if (threadIdx.x >= 64u) {
        /* key wave */
        uint32_t padtail[8];
#pragma unroll
        for (int j = 0; j < 8; j++) padtail[j] = 0u;
        if (MODE == 0) {
            const uint32_t q = e.pwlen >> 2, r = (e.pwlen & 3u) * 8u;
#pragma unroll
            for (int t = 0; t < 8; t++) {
                const uint32_t lo = r ? (p.pad[t] << r) : p.pad[t];
                const uint32_t hi = r ? (p.pad[t] >> (32u - r)) : 0u;
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    if ((uint32_t)j == q + t) padtail[j] |= lo;
                    if ((uint32_t)j == q + t + 1) padtail[j] |= hi;
                }
            }
        }
        uint32_t h[4];
        {
            const uint32_t g0 = base + lane;
            r24_key<MODE, R, NK>(e, p, cs, padw, padtail, g0 < e.count ? g0 : e.count - 1, h);
        }
#pragma unroll 1
        for (uint32_t b = 0; b < nb; b++) {
            __syncthreads();                              /* the RC4 wave is done with batch b-1's S-box */
#pragma unroll
            for (int q = 0; q < 4; q++) keyx[64 * q + lane] = h[q];
            __syncthreads();                              /* batch b's keys are in LDS */
            if (b + 1u < nb) {
                const uint32_t g0 = base + 64u * (b + 1u) + lane;
                r24_key<MODE, R, NK>(e, p, cs, padw, padtail, g0 < e.count ? g0 : e.count - 1, h);
            }
        }
        return;
    }
    /* RC4 wave */
    __builtin_amdgcn_s_setprio(R24_PRIO);
    uint8_t *Sw = S;
    /* the asm KSA needs the S-box area at an LDS address with zero low 16 bits (rc4_ksa_asm); S is this kernel's
     * first LDS object, at 0 -- checked, and a launch that ever breaks it fails loudly instead of computing wrong */
    const uint32_t sbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S);
    if (R24_KSA_ASM && (sbase & 0xffffu) != 0u) {
        if (lane == 0) atomicOr(&R_->pad_, 2u);
        for (uint32_t b = 0; b < nb; b++) { __syncthreads(); __syncthreads(); }   /* keep the key wave's barriers */
        return;
    }
#pragma unroll 1
    for (uint32_t b = 0; b < nb; b++) {
        __syncthreads();
        __syncthreads();
        uint32_t h[4];
#pragma unroll
        for (int q = 0; q < 4; q++) h[q] = keyx[64 * q + lane];
        /* the lane index recomputed here (v_mbcnt, opaque so LLVM cannot hoist base + lane out of the loop): a
         * register holding it across the KSAs was the one value this kernel spilled to scratch */
        uint32_t lid;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lid));
        const uint32_t g = base + 64u * b + lid;
        const bool valid = g < e.count;
        bool ok = false;
        if (R == 2) {
            /* RC4-40 over PAD, compare 32 bytes of U (:161-163, :184-189).  The first 4 keystream bytes decide
             * for all but 2^-32 of the lanes: a wave continues the same keystream (i = 5.., j carried) only
             * when one of its lanes matches U[0:4] */
            uint32_t d[8];
#pragma unroll
            for (int j = 0; j < 8; j++) d[j] = p.pad[j];
            r24_ksa<5>(Sw, sbase, lane, h);
            uint32_t jj = 0;
            rc4_prga_span<1, 4>(Sw, lane << 2, d, jj);
            if (__builtin_amdgcn_ballot_w64(valid && d[0] == p.u[0])) {
                rc4_prga_span<5, 32>(Sw, lane << 2, d, jj);
                ok = true;
#pragma unroll
                for (int j = 0; j < 8; j++) ok = ok && d[j] == p.u[j];
            }
        } else
        /* c = RC4(key, MD5(PAD||ID)); c = RC4(key ^ x, c) for x = 1..19 (:167-174), compare 16 bytes.  Early
         * reject: every pass first produces only 2 keystream bytes and the candidate survives iff c19[0:2]
         * equals U[0:2]; a wave in which some lane survives (2^-16 per lane) redoes its candidates with the full
         * keystream and the reference's complete 16-byte compare (:184-189) */
        for (uint32_t full = 0; full < 2u; full++) {
            uint32_t d[4] = {p.h2[0], p.h2[1], p.h2[2], p.h2[3]};
            /* the asm KSA's key registers, made once per candidate; pass x's key (key ^ x) by XORing x ^ (x - 1)
             * into their byte 0 (16 v_xor per pass, the same count as forming kx and extracting its bytes) */
            uint32_t kb[NK];
            rc4_kb_init<NK>(h, kb);
            for (uint32_t x = 0; x < 20u; x++) {
                if (R24_KSA_ASM) {
                    const uint32_t dx = x ^ (x - 1u);
                    if (x) {
#pragma unroll
                        for (int q = 0; q < NK; q++) kb[q] ^= dx;
                    }
                    rc4_ksa_asm_kb<NK>(sbase, sbase + (lane << 2), kb);
                } else {
                    const uint32_t xx = x * 0x01010101u;
                    uint32_t kx[4] = {h[0] ^ xx, h[1] ^ xx, h[2] ^ xx, h[3] ^ xx};
                    rc4_ksa<NK>(Sw, lane << 2, kx);
                }
                if (full) rc4_prga<16>(Sw, lane << 2, d);
                else rc4_prga<2>(Sw, lane << 2, d);
            }
            if (full) {
                ok = d[0] == p.u[0] && d[1] == p.u[1] && d[2] == p.u[2] && d[3] == p.u[3];
            } else {
                const bool pre = ((d[0] ^ p.u[0]) & 0xffffu) == 0u;
                if (!__builtin_amdgcn_ballot_w64(valid && pre)) break;
            }
        }
        if (valid && ok) report_hit(e, R_, e.start + g, cap, stop_on_first);
    }
}

#endif /* DPRF_PART_PDF */

/* ------------------------------------------------------------------ launchers */
#define GRID(n, b) dim3(((n) + (b) - 1) / (b))

#ifdef DPRF_PART_OFFICE
hipError_t launch_office(const dprf_enum &e, const dprf_office_params &p, const dprf_aes_tables *T,
                         dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s, uint32_t *keys,
                         hipEvent_t mid) {
    if (e.mode == 0) hipLaunchKernelGGL(k_office_kdf<0>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    else if (e.mode == 1) hipLaunchKernelGGL(k_office_kdf<1>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    else hipLaunchKernelGGL(k_office_kdf<2>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    if (mid) (void)hipEventRecord(mid, s);
    hipLaunchKernelGGL(k_office_check, GRID(e.count, 256), dim3(256), 0, s, e, p, T, R, cap, stop, keys);
    return hipGetLastError();
}
#endif

#ifdef DPRF_PART_ODT
hipError_t launch_odt(const dprf_enum &e, const dprf_odt_params &p, const dprf_aes_tables *T,
                      dprf_results *R, uint32_t cap, uint32_t stop, hipStream_t s, uint32_t *keys,
                         hipEvent_t mid) {
    if (e.mode == 0) hipLaunchKernelGGL(k_odt_kdf<0>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    else if (e.mode == 1) hipLaunchKernelGGL(k_odt_kdf<1>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    else hipLaunchKernelGGL(k_odt_kdf<2>, GRID(e.count, 256), dim3(256), 0, s, e, p, R, stop, keys);
    if (mid) (void)hipEventRecord(mid, s);
    hipLaunchKernelGGL(k_odt_check, GRID(e.count, ODT_CHECK_THREADS), dim3(ODT_CHECK_THREADS), 0, s, e, p, T, R, cap, stop, keys);
    return hipGetLastError();
}
#endif /* DPRF_PART_ODT */

#ifdef DPRF_PART_LONG
hipError_t launch_long_prehash(const dprf_enum &e, const dprf_long_params &lp, dprf_results *R, uint32_t cap,
                               uint32_t stop, hipStream_t s) {
    hipLaunchKernelGGL(k_long_prehash, GRID(e.count, 256), dim3(256), 0, s, e, lp, R, cap, stop);
    return hipGetLastError();
}
hipError_t launch_spell_symbols(const dprf_enum &e, const uint32_t *symtab, uint32_t trunc, uint32_t *slots,
                                uint8_t *lens, hipStream_t s) {
    hipLaunchKernelGGL(k_spell_symbols, GRID(e.count, 256), dim3(256), 0, s, e, symtab, trunc, slots, lens);
    return hipGetLastError();
}
#endif

#ifdef DPRF_PART_PDF
hipError_t launch_pdf_r5(const dprf_enum &e, const dprf_pdf_params &p, dprf_results *R, uint32_t cap,
                         uint32_t stop, hipStream_t s) {
#define L5(M, NW, PER) hipLaunchKernelGGL((k_pdf_r5<M, NW, PER>), GRID(e.count, 256 * PER), dim3(256), 0, s, e, p, R, cap, stop)
#define L5W(NW) do { if (R5_PER_MAX >= 16 && e.cslen >= 16) L5(0, NW, 16); else L5(0, NW, 8); } while (0)
    if (e.mode == 0) {
        switch ((e.pwlen + 3u) >> 2) {
        case 0: case 1: L5W(1); break;
        case 2: L5W(2); break;
        case 3: L5W(3); break;
        case 4: L5W(4); break;
        default: L5W(8); break;
        }
    } else if (e.mode == 1 && e.pwlen <= 8) {
        L5(1, 2, 8);
    } else if (e.mode == 1 && e.pwlen <= 16) {
        L5(1, 4, 8);
    } else {
        L5(1, 8, 8);
    }
#undef L5W
#undef L5
    return hipGetLastError();
}
hipError_t launch_pdf_r24(const dprf_enum &e, const dprf_pdf_params &p, dprf_results *R, uint32_t cap,
                          uint32_t stop, hipStream_t s) {
#define L24(M, RR, NK) hipLaunchKernelGGL((k_pdf_r24<M, RR, NK>), GRID(e.count, 64 * r24_batches<RR>::v), dim3(128), 0, s, e, p, R, cap, stop)
    if (p.R == 2) { if (e.mode == 0) L24(0, 2, 5); else L24(1, 2, 5); }
    else if (p.n == 16) { if (e.mode == 0) L24(0, 3, 16); else L24(1, 3, 16); }
    else { if (e.mode == 0) L24(0, 3, 5); else L24(1, 3, 5); }
#undef L24
    return hipGetLastError();
}
#endif /* DPRF_PART_PDF */

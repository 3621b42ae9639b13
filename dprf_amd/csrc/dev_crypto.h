/* dev_crypto.h -- gfx950 device primitives for the verification kernels.
 *
 * Everything here is one-candidate-per-lane VALU code: hash state lives in VGPRs, loops are fully
 * unrolled so every message-word index is static (runtime-indexed register arrays would spill to
 * scratch), and constant message words are left as C constants so LLVM folds them out of the
 * schedule.  gfx950-specific: v_bitop3_b32 (any 3-input boolean function in one instruction) for
 * Ch/Maj/parity/XOR3, v_alignbit_b32 for rotates, v_add3_u32 for the additions, v_perm_b32 for byte
 * shuffles.
 *
 * Algorithms are from the standards (FIPS 180-4, RFC 1321, FIPS 197); the reference reaches them
 * through OpenSSL.
 */
#ifndef DPRF_DEV_CRYPTO_H
#define DPRF_DEV_CRYPTO_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEVI __device__ __forceinline__

/* ------------------------------------------------------------------ bit helpers */
DEVI uint32_t rol32(uint32_t x, int s) { return __builtin_rotateleft32(x, s); }
DEVI uint32_t ror32(uint32_t x, int s) { return __builtin_rotateright32(x, s); }
DEVI uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

/* v_bitop3_b32 truth tables: src0 <-> 0xF0, src1 <-> 0xCC, src2 <-> 0xAA. */
#define LUT_XOR3 0x96
#define LUT_CH 0xCA   /* (a & b) | (~a & c) */
#define LUT_MAJ 0xE8  /* (a & b) | (a & c) | (b & c) */
#define LUT_MD5_I 0x39 /* I(b,c,d) = c ^ (b | ~d) */

/* Use bitop3 only when no operand is a compile-time constant, so that constant message words (zeros
 * of SHA padding, etc.) still fold away in plain XOR form. */
#define CONSTP(x) __builtin_constant_p(x)
DEVI uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    if (CONSTP(a) || CONSTP(b) || CONSTP(c)) return a ^ b ^ c;
    return __builtin_amdgcn_bitop3_b32(a, b, c, LUT_XOR3);
}
DEVI uint32_t f_ch(uint32_t a, uint32_t b, uint32_t c) {
    if (CONSTP(a) && CONSTP(b) && CONSTP(c)) return (a & b) | (~a & c);
    return __builtin_amdgcn_bitop3_b32(a, b, c, LUT_CH);
}
DEVI uint32_t f_maj(uint32_t a, uint32_t b, uint32_t c) {
    if (CONSTP(a) && CONSTP(b) && CONSTP(c)) return (a & b) | (a & c) | (b & c);
    return __builtin_amdgcn_bitop3_b32(a, b, c, LUT_MAJ);
}
DEVI uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

/* ------------------------------------------------------------------ SHA-1 (FIPS 180-4 6.1.2) */
#define SHA1_IV0 0x67452301u
#define SHA1_IV1 0xEFCDAB89u
#define SHA1_IV2 0x98BADCFEu
#define SHA1_IV3 0x10325476u
#define SHA1_IV4 0xC3D2E1F0u

/* One compression, 16-word rolling schedule.  st: chaining value in/out, w: message (clobbered). */
DEVI void sha1_compress(uint32_t st[5], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#pragma unroll
    for (int t = 0; t < 80; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rol32(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20)      { f = f_ch(b, c, d);  k = 0x5A827999u; }
        else if (t < 40) { f = xor3(b, c, d);  k = 0x6ED9EBA1u; }
        else if (t < 60) { f = f_maj(b, c, d); k = 0x8F1BBCDCu; }
        else             { f = xor3(b, c, d);  k = 0xCA62C1D6u; }
        uint32_t tmp = rol32(a, 5) + f + e + (k + wt);
        e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}
/* SHA-1 from a fixed starting state (PBKDF2's HMAC midstates: the same for all 1,023 iterations of a candidate).
 * sha1_pre computes, once per candidate, everything of rounds 0-4 that does not depend on the message: round 0's
 * whole sum but w0, round 1's f + e + k as ONE value (LLVM hoists f and e + k as two), and e + k of rounds 2-4.  They
 * leave through an empty asm so that LLVM cannot re-split them inside the loop.  2,070 -> 2,062 issue slots per
 * PBKDF2 iteration (tools/asm_slots.py); the extra live values need more than the 64 VGPRs of 8 waves per SIMD
 * (k_odt_kdf runs at ODT_KDF_WAVES). */
struct sha1_pre_t { uint32_t p0, p1, p2, p3, p4, ra, rb; };
DEVI sha1_pre_t sha1_pre(const uint32_t st[5]) {
    const uint32_t K = 0x5A827999u, A = st[0], B = st[1], C = st[2], D = st[3], E = st[4];
    sha1_pre_t P;
    P.ra = rol32(A, 30);
    P.rb = rol32(B, 30);
    P.p0 = rol32(A, 5) + f_ch(B, C, D) + E + K;
    P.p1 = f_ch(A, P.rb, C) + D + K;
    P.p2 = C + K;
    P.p3 = P.rb + K;
    P.p4 = P.ra + K;
    asm volatile("" : "+v"(P.p0), "+v"(P.p1), "+v"(P.p2), "+v"(P.p3), "+v"(P.p4));
    return P;
}
/* st: the fixed starting state, out = st + the compression of w (w is overwritten by the schedule) */
DEVI void sha1_compress_pre(const uint32_t st[5], const sha1_pre_t &P, uint32_t w[16], uint32_t out[5]) {
    const uint32_t K = 0x5A827999u;
    const uint32_t a1 = P.p0 + w[0];
    const uint32_t a2 = rol32(a1, 5) + P.p1 + w[1];
    const uint32_t a3 = rol32(a2, 5) + f_ch(a1, P.ra, P.rb) + P.p2 + w[2];
    const uint32_t r1 = rol32(a1, 30);
    const uint32_t a4 = rol32(a3, 5) + f_ch(a2, r1, P.ra) + P.p3 + w[3];
    const uint32_t r2 = rol32(a2, 30);
    const uint32_t a5 = rol32(a4, 5) + f_ch(a3, r2, r1) + P.p4 + w[4];
    uint32_t a = a5, b = a4, c = rol32(a3, 30), d = r2, e = r1;
#pragma unroll
    for (int t = 5; t < 80; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = rol32(xor3(w[(t - 3) & 15], w[(t - 8) & 15], w[(t - 14) & 15]) ^ w[t & 15], 1);
            w[t & 15] = wt;
        }
        uint32_t f, k;
        if (t < 20)      { f = f_ch(b, c, d);  k = K; }
        else if (t < 40) { f = xor3(b, c, d);  k = 0x6ED9EBA1u; }
        else if (t < 60) { f = f_maj(b, c, d); k = 0x8F1BBCDCu; }
        else             { f = xor3(b, c, d);  k = 0xCA62C1D6u; }
        const uint32_t tmp = rol32(a, 5) + f + e + (k + wt);
        e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
    }
    out[0] = st[0] + a; out[1] = st[1] + b; out[2] = st[2] + c; out[3] = st[3] + d; out[4] = st[4] + e;
}
DEVI void sha1_iv(uint32_t st[5]) {
    st[0] = SHA1_IV0; st[1] = SHA1_IV1; st[2] = SHA1_IV2; st[3] = SHA1_IV3; st[4] = SHA1_IV4;
}

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4 6.2.2) */
/* the round constants as a constexpr function so the unrolled code gets literals, not loads */
DEVI constexpr uint32_t k256(int t) {
    constexpr uint32_t K[64] = {
    0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
    0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
    0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
    0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
    0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
    0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
    0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
    0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
    return K[t];
}

DEVI void sha256_iv(uint32_t st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}
DEVI uint32_t S0_256(uint32_t a) { return xor3(ror32(a, 2), ror32(a, 13), ror32(a, 22)); }
DEVI uint32_t S1_256(uint32_t e) { return xor3(ror32(e, 6), ror32(e, 11), ror32(e, 25)); }
DEVI uint32_t s0_256(uint32_t x) { return xor3(ror32(x, 7), ror32(x, 18), x >> 3); }
DEVI uint32_t s1_256(uint32_t x) { return xor3(ror32(x, 17), ror32(x, 19), x >> 10); }

DEVI void sha256_compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
        uint32_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            wt = w[t & 15] + s0_256(w[(t - 15) & 15]) + w[(t - 7) & 15] + s1_256(w[(t - 2) & 15]);
            w[t & 15] = wt;
        }
        uint32_t t1 = h + S1_256(e) + f_ch(e, f, g) + (k256(t) + wt);
        uint32_t t2 = S0_256(a) + f_maj(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* ------------------------------------------------------------------ SHA-512 / SHA-384 (FIPS 180-4 6.4) */
DEVI constexpr uint64_t k512(int t) {
    constexpr uint64_t K[80] = {
    0x428a2f98d728ae22ull,0x7137449123ef65cdull,0xb5c0fbcfec4d3b2full,0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull,0x59f111f1b605d019ull,0x923f82a4af194f9bull,0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull,0x12835b0145706fbeull,0x243185be4ee4b28cull,0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full,0x80deb1fe3b1696b1ull,0x9bdc06a725c71235ull,0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull,0xefbe4786384f25e3ull,0x0fc19dc68b8cd5b5ull,0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull,0x4a7484aa6ea6e483ull,0x5cb0a9dcbd41fbd4ull,0x76f988da831153b5ull,
    0x983e5152ee66dfabull,0xa831c66d2db43210ull,0xb00327c898fb213full,0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull,0xd5a79147930aa725ull,0x06ca6351e003826full,0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull,0x2e1b21385c26c926ull,0x4d2c6dfc5ac42aedull,0x53380d139d95b3dfull,
    0x650a73548baf63deull,0x766a0abb3c77b2a8ull,0x81c2c92e47edaee6ull,0x92722c851482353bull,
    0xa2bfe8a14cf10364ull,0xa81a664bbc423001ull,0xc24b8b70d0f89791ull,0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull,0xd69906245565a910ull,0xf40e35855771202aull,0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull,0x1e376c085141ab53ull,0x2748774cdf8eeb99ull,0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull,0x4ed8aa4ae3418acbull,0x5b9cca4f7763e373ull,0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull,0x78a5636f43172f60ull,0x84c87814a1f0ab72ull,0x8cc702081a6439ecull,
    0x90befffa23631e28ull,0xa4506cebde82bde9ull,0xbef9a3f7b2c67915ull,0xc67178f2e372532bull,
    0xca273eceea26619cull,0xd186b8c721c0c207ull,0xeada7dd6cde0eb1eull,0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull,0x0a637dc5a2c898a6ull,0x113f9804bef90daeull,0x1b710b35131c471bull,
    0x28db77f523047d84ull,0x32caab7b40c72493ull,0x3c9ebe0a15c9bebcull,0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull,0x597f299cfc657e2aull,0x5fcb6fab3ad6faecull,0x6c44198c4a475817ull};
    return K[t];
}
/* 64-bit values are VGPR pairs built from two 32-bit halves with a bit-cast (no arithmetic: the pair is
 * just a REG_SEQUENCE).  Rotates / shifts work on the halves with v_alignbit_b32 (2 slots each; the
 * compiler's own v_lshrrev_b64 costs 4.6), and every 64-bit addition is ONE v_lshl_add_u64 in inline asm
 * (2.6 slots, tools/valu_peak.hip): written as plain `+` on a value assembled as (hi << 32) | lo, LLVM
 * split each add into two v_lshl_add_u64 of the zero-extended halves plus two v_mov -- 1,202 instead of
 * ~760 adds and 453 moves per SHA-512 compression (8,444 -> ~6,800 slots). */
DEVI uint64_t pack64(uint32_t hi, uint32_t lo) { return __builtin_bit_cast(uint64_t, make_uint2(lo, hi)); }
DEVI uint32_t lo32(uint64_t x) { return __builtin_bit_cast(uint2, x).x; }
DEVI uint32_t hi32(uint64_t x) { return __builtin_bit_cast(uint2, x).y; }
DEVI uint64_t add64(uint64_t a, uint64_t b) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
/* a + k for a compile-time constant k: the constant goes in an SGPR pair (SALU s_mov, no VALU slot) */
DEVI uint64_t add64k(uint64_t a, uint64_t k) {
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(a), "s"(k));
    return r;
}
DEVI uint64_t ror64(uint64_t x, int s) {
    const uint32_t lo = lo32(x), hi = hi32(x);
    if (s == 32) return pack64(lo, hi);
    if (s < 32) return pack64(__builtin_amdgcn_alignbit(lo, hi, s), __builtin_amdgcn_alignbit(hi, lo, s));
    return pack64(__builtin_amdgcn_alignbit(hi, lo, s - 32), __builtin_amdgcn_alignbit(lo, hi, s - 32));
}
DEVI uint64_t shr64(uint64_t x, int s) {   /* 0 < s < 32 */
    const uint32_t lo = lo32(x), hi = hi32(x);
    return pack64(hi >> s, __builtin_amdgcn_alignbit(hi, lo, s));
}
DEVI uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
    return pack64(xor3(hi32(a), hi32(b), hi32(c)), xor3(lo32(a), lo32(b), lo32(c)));
}
DEVI uint64_t ch64(uint64_t a, uint64_t b, uint64_t c) {
    return pack64(f_ch(hi32(a), hi32(b), hi32(c)), f_ch(lo32(a), lo32(b), lo32(c)));
}
DEVI uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
    return pack64(f_maj(hi32(a), hi32(b), hi32(c)), f_maj(lo32(a), lo32(b), lo32(c)));
}
DEVI void sha512_iv(uint64_t st[8], bool is384) {
    if (is384) {
        st[0] = 0xcbbb9d5dc1059ed8ull; st[1] = 0x629a292a367cd507ull; st[2] = 0x9159015a3070dd17ull;
        st[3] = 0x152fecd8f70e5939ull; st[4] = 0x67332667ffc00b31ull; st[5] = 0x8eb44a8768581511ull;
        st[6] = 0xdb0c2e0d64f98fa7ull; st[7] = 0x47b5481dbefa4fa4ull;
    } else {
        st[0] = 0x6a09e667f3bcc908ull; st[1] = 0xbb67ae8584caa73bull; st[2] = 0x3c6ef372fe94f82bull;
        st[3] = 0xa54ff53a5f1d36f1ull; st[4] = 0x510e527fade682d1ull; st[5] = 0x9b05688c2b3e6c1full;
        st[6] = 0x1f83d9abfb41bd6bull; st[7] = 0x5be0cd19137e2179ull;
    }
}
DEVI void sha512_compress(uint64_t st[8], uint64_t w[16]) {
    uint64_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma clang loop unroll(full)
    for (int t = 0; t < 80; t++) {
        uint64_t wt;
        if (t < 16) {
            wt = w[t];
        } else {
            const uint64_t x = w[(t - 15) & 15], y = w[(t - 2) & 15];
            const uint64_t s0 = xor3_64(ror64(x, 1), ror64(x, 8), shr64(x, 7));
            const uint64_t s1 = xor3_64(ror64(y, 19), ror64(y, 61), shr64(y, 6));
            wt = add64(add64(w[t & 15], s0), add64(w[(t - 7) & 15], s1));
            w[t & 15] = wt;
        }
        const uint64_t S1 = xor3_64(ror64(e, 14), ror64(e, 18), ror64(e, 41));
        const uint64_t t1 = add64(add64(h, S1), add64(ch64(e, f, g), add64k(wt, k512(t))));
        const uint64_t S0 = xor3_64(ror64(a, 28), ror64(a, 34), ror64(a, 39));
        const uint64_t t2 = add64(S0, maj64(a, b, c));
        h = g; g = f; f = e; e = add64(d, t1); d = c; c = b; b = a; a = add64(t1, t2);
    }
    st[0] = add64(st[0], a); st[1] = add64(st[1], b); st[2] = add64(st[2], c); st[3] = add64(st[3], d);
    st[4] = add64(st[4], e); st[5] = add64(st[5], f); st[6] = add64(st[6], g); st[7] = add64(st[7], h);
}

/* ------------------------------------------------------------------ MD5 (RFC 1321 3.4) */
DEVI constexpr uint32_t kmd5(int i) {
    constexpr uint32_t K[64] = {
    0xd76aa478u,0xe8c7b756u,0x242070dbu,0xc1bdceeeu,0xf57c0fafu,0x4787c62au,0xa8304613u,0xfd469501u,
    0x698098d8u,0x8b44f7afu,0xffff5bb1u,0x895cd7beu,0x6b901122u,0xfd987193u,0xa679438eu,0x49b40821u,
    0xf61e2562u,0xc040b340u,0x265e5a51u,0xe9b6c7aau,0xd62f105du,0x02441453u,0xd8a1e681u,0xe7d3fbc8u,
    0x21e1cde6u,0xc33707d6u,0xf4d50d87u,0x455a14edu,0xa9e3e905u,0xfcefa3f8u,0x676f02d9u,0x8d2a4c8au,
    0xfffa3942u,0x8771f681u,0x6d9d6122u,0xfde5380cu,0xa4beea44u,0x4bdecfa9u,0xf6bb4b60u,0xbebfbc70u,
    0x289b7ec6u,0xeaa127fau,0xd4ef3085u,0x04881d05u,0xd9d4d039u,0xe6db99e5u,0x1fa27cf8u,0xc4ac5665u,
    0xf4292244u,0x432aff97u,0xab9423a7u,0xfc93a039u,0x655b59c3u,0x8f0ccc92u,0xffeff47du,0x85845dd1u,
    0x6fa87e4fu,0xfe2ce6e0u,0xa3014314u,0x4e0811a1u,0xf7537e82u,0xbd3af235u,0x2ad7d2bbu,0xeb86d391u};
    return K[i];
}
DEVI constexpr int smd5(int i) {
    constexpr int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    return S[(i >> 4) * 4 + (i & 3)];
}
DEVI void md5_iv(uint32_t st[4]) { st[0] = 0x67452301u; st[1] = 0xefcdab89u; st[2] = 0x98badcfeu; st[3] = 0x10325476u; }
DEVI void md5_compress(uint32_t st[4], const uint32_t m[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        uint32_t f; int g;
        if (i < 16)      { f = f_ch(b, c, d);  g = i; }
        else if (i < 32) { f = f_ch(d, b, c);  g = (5 * i + 1) & 15; }
        else if (i < 48) { f = xor3(b, c, d);  g = (3 * i + 5) & 15; }
        else {
            /* I(b,c,d) = c ^ (b | ~d) */
            if (CONSTP(b) && CONSTP(c) && CONSTP(d)) f = c ^ (b | ~d);
            else f = __builtin_amdgcn_bitop3_b32(b, c, d, LUT_MD5_I);
            g = (7 * i) & 15;
        }
        uint32_t tmp = d; d = c; c = b;
        b = b + rol32(a + f + (kmd5(i) + m[g]), smd5(i));
        a = tmp;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
}

/* ------------------------------------------------------------------ message packing helpers
 * Candidate bytes are held LE-packed in 16 words (byte k in word k>>2, bits 8*(k&3)).  These build
 * padded hash blocks for a runtime length with static word indices only. */

/* byte mask of the first `len - 4*j` bytes of word j (LE), clamped to 0..4 bytes */
DEVI uint32_t le_keep_mask(int j, uint32_t len) {
    int n = (int)len - 4 * j;
    return n <= 0 ? 0u : (n >= 4 ? 0xffffffffu : ((1u << (8 * n)) - 1u));
}
/* 0x80 at byte position len if it falls in word j (LE), else 0 */
DEVI uint32_t le_pad80(int j, uint32_t len) {
    int n = (int)len - 4 * j;
    return (n >= 0 && n < 4) ? (0x80u << (8 * n)) : 0u;
}

/* ------------------------------------------------------------------ AES with LDS T-tables
 * te/td: 256-entry BE-column tables in LDS; sb/isb: S-box and inverse S-box bytes in LDS.
 * Te1..3 / Td1..3 are byte rotations of Te0 / Td0 (v_alignbit), saving 3 KB of LDS per table. */
struct aes_lds {
    uint32_t te[256];
    uint32_t td[256];
    uint32_t sb[64];   /* S-box bytes packed 4 per word */
    uint32_t isb[64];
};

DEVI uint32_t lds_byte(const uint32_t *tab, uint32_t idx) {
    return ((const uint8_t *)tab)[idx];
}
DEVI uint32_t T0(const uint32_t *t, uint32_t x) { return t[x]; }
DEVI uint32_t T1(const uint32_t *t, uint32_t x) { return ror32(t[x], 8); }
DEVI uint32_t T2(const uint32_t *t, uint32_t x) { return ror32(t[x], 16); }
DEVI uint32_t T3(const uint32_t *t, uint32_t x) { return ror32(t[x], 24); }
#define B3(x) ((x) >> 24)
#define B2(x) (((x) >> 16) & 0xffu)
#define B1(x) (((x) >> 8) & 0xffu)
#define B0(x) ((x) & 0xffu)

/* SubWord of a BE word through the S-box */
DEVI uint32_t aes_subword(const aes_lds &L, uint32_t x) {
    return (lds_byte(L.sb, B3(x)) << 24) | (lds_byte(L.sb, B2(x)) << 16) | (lds_byte(L.sb, B1(x)) << 8) |
           lds_byte(L.sb, B0(x));
}

/* AES-128 forward key schedule, rk[44] BE words (FIPS 197 5.2) */
DEVI void aes128_expand(const aes_lds &L, const uint32_t key[4], uint32_t rk[44]) {
    const uint32_t rcon[10] = {0x01000000u, 0x02000000u, 0x04000000u, 0x08000000u, 0x10000000u,
                               0x20000000u, 0x40000000u, 0x80000000u, 0x1b000000u, 0x36000000u};
    rk[0] = key[0]; rk[1] = key[1]; rk[2] = key[2]; rk[3] = key[3];
#pragma unroll
    for (int i = 0; i < 10; i++) {
        uint32_t t = rk[4 * i + 3];
        rk[4 * i + 4] = rk[4 * i] ^ aes_subword(L, rol32(t, 8)) ^ rcon[i];
        rk[4 * i + 5] = rk[4 * i + 1] ^ rk[4 * i + 4];
        rk[4 * i + 6] = rk[4 * i + 2] ^ rk[4 * i + 5];
        rk[4 * i + 7] = rk[4 * i + 3] ^ rk[4 * i + 6];
    }
}
/* AES-256 forward key schedule, rk[60] */
DEVI void aes256_expand(const aes_lds &L, const uint32_t key[8], uint32_t rk[60]) {
    const uint32_t rcon[7] = {0x01000000u, 0x02000000u, 0x04000000u, 0x08000000u, 0x10000000u,
                              0x20000000u, 0x40000000u};
#pragma unroll
    for (int i = 0; i < 8; i++) rk[i] = key[i];
#pragma unroll
    for (int i = 8; i < 60; i++) {
        uint32_t t = rk[i - 1];
        if (i % 8 == 0) t = aes_subword(L, rol32(t, 8)) ^ rcon[i / 8 - 1];
        else if (i % 8 == 4) t = aes_subword(L, t);
        rk[i] = rk[i - 8] ^ t;
    }
}
/* InvMixColumns of a round-key word: Td0[S[b3]] ^ Td1[S[b2]] ^ Td2[S[b1]] ^ Td3[S[b0]] */
DEVI uint32_t aes_imc(const aes_lds &L, uint32_t w) {
    return xor3(T0(L.td, lds_byte(L.sb, B3(w))), T1(L.td, lds_byte(L.sb, B2(w))), T2(L.td, lds_byte(L.sb, B1(w)))) ^
           T3(L.td, lds_byte(L.sb, B0(w)));
}
/* Equivalent-inverse-cipher decryption schedule dk from forward rk (nr rounds), in place. */
template <int NR>
DEVI void aes_dec_schedule(const aes_lds &L, const uint32_t rk[4 * (NR + 1)], uint32_t dk[4 * (NR + 1)]) {
#pragma unroll
    for (int r = 0; r <= NR; r++) {
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t w = rk[4 * (NR - r) + c];
            dk[4 * r + c] = (r == 0 || r == NR) ? w : aes_imc(L, w);
        }
    }
}
template <int NR>
DEVI void aes_encrypt(const aes_lds &L, const uint32_t *rk, const uint32_t in[4], uint32_t out[4]) {
    uint32_t s0 = in[0] ^ rk[0], s1 = in[1] ^ rk[1], s2 = in[2] ^ rk[2], s3 = in[3] ^ rk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t0 = xor3(xor3(T0(L.te, B3(s0)), T1(L.te, B2(s1)), T2(L.te, B1(s2))), T3(L.te, B0(s3)), rk[4 * r + 0]);
        uint32_t t1 = xor3(xor3(T0(L.te, B3(s1)), T1(L.te, B2(s2)), T2(L.te, B1(s3))), T3(L.te, B0(s0)), rk[4 * r + 1]);
        uint32_t t2 = xor3(xor3(T0(L.te, B3(s2)), T1(L.te, B2(s3)), T2(L.te, B1(s0))), T3(L.te, B0(s1)), rk[4 * r + 2]);
        uint32_t t3 = xor3(xor3(T0(L.te, B3(s3)), T1(L.te, B2(s0)), T2(L.te, B1(s1))), T3(L.te, B0(s2)), rk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t *r = rk + 4 * NR;
    out[0] = ((lds_byte(L.sb, B3(s0)) << 24) | (lds_byte(L.sb, B2(s1)) << 16) | (lds_byte(L.sb, B1(s2)) << 8) | lds_byte(L.sb, B0(s3))) ^ r[0];
    out[1] = ((lds_byte(L.sb, B3(s1)) << 24) | (lds_byte(L.sb, B2(s2)) << 16) | (lds_byte(L.sb, B1(s3)) << 8) | lds_byte(L.sb, B0(s0))) ^ r[1];
    out[2] = ((lds_byte(L.sb, B3(s2)) << 24) | (lds_byte(L.sb, B2(s3)) << 16) | (lds_byte(L.sb, B1(s0)) << 8) | lds_byte(L.sb, B0(s1))) ^ r[2];
    out[3] = ((lds_byte(L.sb, B3(s3)) << 24) | (lds_byte(L.sb, B2(s0)) << 16) | (lds_byte(L.sb, B1(s1)) << 8) | lds_byte(L.sb, B0(s2))) ^ r[3];
}
template <int NR>
DEVI void aes_decrypt(const aes_lds &L, const uint32_t *dk, const uint32_t in[4], uint32_t out[4]) {
    uint32_t s0 = in[0] ^ dk[0], s1 = in[1] ^ dk[1], s2 = in[2] ^ dk[2], s3 = in[3] ^ dk[3];
#pragma unroll
    for (int r = 1; r < NR; r++) {
        uint32_t t0 = xor3(xor3(T0(L.td, B3(s0)), T1(L.td, B2(s3)), T2(L.td, B1(s2))), T3(L.td, B0(s1)), dk[4 * r + 0]);
        uint32_t t1 = xor3(xor3(T0(L.td, B3(s1)), T1(L.td, B2(s0)), T2(L.td, B1(s3))), T3(L.td, B0(s2)), dk[4 * r + 1]);
        uint32_t t2 = xor3(xor3(T0(L.td, B3(s2)), T1(L.td, B2(s1)), T2(L.td, B1(s0))), T3(L.td, B0(s3)), dk[4 * r + 2]);
        uint32_t t3 = xor3(xor3(T0(L.td, B3(s3)), T1(L.td, B2(s2)), T2(L.td, B1(s1))), T3(L.td, B0(s0)), dk[4 * r + 3]);
        s0 = t0; s1 = t1; s2 = t2; s3 = t3;
    }
    const uint32_t *r = dk + 4 * NR;
    out[0] = ((lds_byte(L.isb, B3(s0)) << 24) | (lds_byte(L.isb, B2(s3)) << 16) | (lds_byte(L.isb, B1(s2)) << 8) | lds_byte(L.isb, B0(s1))) ^ r[0];
    out[1] = ((lds_byte(L.isb, B3(s1)) << 24) | (lds_byte(L.isb, B2(s0)) << 16) | (lds_byte(L.isb, B1(s3)) << 8) | lds_byte(L.isb, B0(s2))) ^ r[1];
    out[2] = ((lds_byte(L.isb, B3(s2)) << 24) | (lds_byte(L.isb, B2(s1)) << 16) | (lds_byte(L.isb, B1(s0)) << 8) | lds_byte(L.isb, B0(s3))) ^ r[2];
    out[3] = ((lds_byte(L.isb, B3(s3)) << 24) | (lds_byte(L.isb, B2(s2)) << 16) | (lds_byte(L.isb, B1(s1)) << 8) | lds_byte(L.isb, B0(s0))) ^ r[3];
}

#endif

/* oracle.c -- CPU restatement of the reference verifiers.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Primitives are written from their standards (FIPS 180-4 SHA-1/SHA-2, RFC 1321 MD5, FIPS 197 AES,
 * RC4 as in RFC 6229's test vectors, RFC 8018 PBKDF2) and pinned by KATs in tests/test_oracle_kat.py.
 * The verify functions restate the reference line by line (citations inline), including its quirks
 * (SURVEY.md Appendix B).  Speed is secondary; clarity is the point.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ work counters */
static __thread uint64_t g_cnt[ORC_NCOUNT];
#define CNT(i) (g_cnt[(i)]++)

static inline uint32_t rol32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }
static inline uint32_t ror32(uint32_t x, int s) { return (x >> s) | (x << (32 - s)); }
static inline uint64_t ror64(uint64_t x, int s) { return (x >> s) | (x << (64 - s)); }
static inline uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static inline uint32_t le32(const uint8_t *p) {
    return ((uint32_t)p[3] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[1] << 8) | p[0];
}
static inline uint64_t be64(const uint8_t *p) { return ((uint64_t)be32(p) << 32) | be32(p + 4); }
static inline void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
}
static inline void put_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void put_be64(uint8_t *p, uint64_t v) { put_be32(p, (uint32_t)(v >> 32)); put_be32(p + 4, (uint32_t)v); }

/* ------------------------------------------------------------------ SHA-1 (FIPS 180-4 6.1) */
typedef struct { uint32_t h[5]; uint8_t buf[64]; size_t nbuf; uint64_t total; } sha1_t;

static void sha1_compress(uint32_t h[5], const uint8_t blk[64]) {
    uint32_t w[80];
    CNT(0);
    for (int t = 0; t < 16; t++) w[t] = be32(blk + 4 * t);
    for (int t = 16; t < 80; t++) w[t] = rol32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
        uint32_t f, k;
        if (t < 20)      { f = (b & c) | (~b & d);           k = 0x5A827999u; }
        else if (t < 40) { f = b ^ c ^ d;                    k = 0x6ED9EBA1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d);  k = 0x8F1BBCDCu; }
        else             { f = b ^ c ^ d;                    k = 0xCA62C1D6u; }
        uint32_t tmp = rol32(a, 5) + f + e + k + w[t];
        e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}
static void sha1_init(sha1_t *s) {
    static const uint32_t iv[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    memcpy(s->h, iv, sizeof iv); s->nbuf = 0; s->total = 0;
}
static void sha1_update(sha1_t *s, const uint8_t *m, size_t n) {
    s->total += n;
    while (n) {
        size_t k = 64 - s->nbuf; if (k > n) k = n;
        memcpy(s->buf + s->nbuf, m, k); s->nbuf += k; m += k; n -= k;
        if (s->nbuf == 64) { sha1_compress(s->h, s->buf); s->nbuf = 0; }
    }
}
static void sha1_final(sha1_t *s, uint8_t out[20]) {
    uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0, len[8];
    sha1_update(s, &pad, 1);
    while (s->nbuf != 56) sha1_update(s, &z, 1);
    put_be64(len, bits); sha1_update(s, len, 8);
    for (int i = 0; i < 5; i++) put_be32(out + 4 * i, s->h[i]);
}
void orc_sha1(const uint8_t *m, size_t n, uint8_t out[20]) {
    sha1_t s; sha1_init(&s); sha1_update(&s, m, n); sha1_final(&s, out);
}

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4 6.2) */
static const uint32_t K256[64] = {
    0x428a2f98u,0x71374491u,0xb5c0fbcfu,0xe9b5dba5u,0x3956c25bu,0x59f111f1u,0x923f82a4u,0xab1c5ed5u,
    0xd807aa98u,0x12835b01u,0x243185beu,0x550c7dc3u,0x72be5d74u,0x80deb1feu,0x9bdc06a7u,0xc19bf174u,
    0xe49b69c1u,0xefbe4786u,0x0fc19dc6u,0x240ca1ccu,0x2de92c6fu,0x4a7484aau,0x5cb0a9dcu,0x76f988dau,
    0x983e5152u,0xa831c66du,0xb00327c8u,0xbf597fc7u,0xc6e00bf3u,0xd5a79147u,0x06ca6351u,0x14292967u,
    0x27b70a85u,0x2e1b2138u,0x4d2c6dfcu,0x53380d13u,0x650a7354u,0x766a0abbu,0x81c2c92eu,0x92722c85u,
    0xa2bfe8a1u,0xa81a664bu,0xc24b8b70u,0xc76c51a3u,0xd192e819u,0xd6990624u,0xf40e3585u,0x106aa070u,
    0x19a4c116u,0x1e376c08u,0x2748774cu,0x34b0bcb5u,0x391c0cb3u,0x4ed8aa4au,0x5b9cca4fu,0x682e6ff3u,
    0x748f82eeu,0x78a5636fu,0x84c87814u,0x8cc70208u,0x90befffau,0xa4506cebu,0xbef9a3f7u,0xc67178f2u};
typedef struct { uint32_t h[8]; uint8_t buf[64]; size_t nbuf; uint64_t total; } sha256_t;

static void sha256_compress(uint32_t h[8], const uint8_t blk[64]) {
    uint32_t w[64];
    CNT(1);
    for (int t = 0; t < 16; t++) w[t] = be32(blk + 4 * t);
    for (int t = 16; t < 64; t++) {
        uint32_t s0 = ror32(w[t - 15], 7) ^ ror32(w[t - 15], 18) ^ (w[t - 15] >> 3);
        uint32_t s1 = ror32(w[t - 2], 17) ^ ror32(w[t - 2], 19) ^ (w[t - 2] >> 10);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 64; t++) {
        uint32_t S1 = ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = hh + S1 + ch + K256[t] + w[t];
        uint32_t S0 = ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha256_init(sha256_t *s) {
    static const uint32_t iv[8] = {0x6a09e667u,0xbb67ae85u,0x3c6ef372u,0xa54ff53au,
                                   0x510e527fu,0x9b05688cu,0x1f83d9abu,0x5be0cd19u};
    memcpy(s->h, iv, sizeof iv); s->nbuf = 0; s->total = 0;
}
static void sha256_update(sha256_t *s, const uint8_t *m, size_t n) {
    s->total += n;
    while (n) {
        size_t k = 64 - s->nbuf; if (k > n) k = n;
        memcpy(s->buf + s->nbuf, m, k); s->nbuf += k; m += k; n -= k;
        if (s->nbuf == 64) { sha256_compress(s->h, s->buf); s->nbuf = 0; }
    }
}
static void sha256_final(sha256_t *s, uint8_t out[32]) {
    uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0, len[8];
    sha256_update(s, &pad, 1);
    while (s->nbuf != 56) sha256_update(s, &z, 1);
    put_be64(len, bits); sha256_update(s, len, 8);
    for (int i = 0; i < 8; i++) put_be32(out + 4 * i, s->h[i]);
}
void orc_sha256(const uint8_t *m, size_t n, uint8_t out[32]) {
    sha256_t s; sha256_init(&s); sha256_update(&s, m, n); sha256_final(&s, out);
}

/* ------------------------------------------------------------------ SHA-512 / SHA-384 (FIPS 180-4 6.4/6.5) */
static const uint64_t K512[80] = {
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
typedef struct { uint64_t h[8]; uint8_t buf[128]; size_t nbuf; uint64_t total; } sha512_t;

static void sha512_compress(uint64_t h[8], const uint8_t blk[128]) {
    uint64_t w[80];
    CNT(2);
    for (int t = 0; t < 16; t++) w[t] = be64(blk + 8 * t);
    for (int t = 16; t < 80; t++) {
        uint64_t s0 = ror64(w[t - 15], 1) ^ ror64(w[t - 15], 8) ^ (w[t - 15] >> 7);
        uint64_t s1 = ror64(w[t - 2], 19) ^ ror64(w[t - 2], 61) ^ (w[t - 2] >> 6);
        w[t] = w[t - 16] + s0 + w[t - 7] + s1;
    }
    uint64_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
    for (int t = 0; t < 80; t++) {
        uint64_t S1 = ror64(e, 14) ^ ror64(e, 18) ^ ror64(e, 41);
        uint64_t ch = (e & f) ^ (~e & g);
        uint64_t t1 = hh + S1 + ch + K512[t] + w[t];
        uint64_t S0 = ror64(a, 28) ^ ror64(a, 34) ^ ror64(a, 39);
        uint64_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint64_t t2 = S0 + mj;
        hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
static void sha512_init_iv(sha512_t *s, int is384) {
    static const uint64_t iv512[8] = {0x6a09e667f3bcc908ull,0xbb67ae8584caa73bull,0x3c6ef372fe94f82bull,
        0xa54ff53a5f1d36f1ull,0x510e527fade682d1ull,0x9b05688c2b3e6c1full,0x1f83d9abfb41bd6bull,
        0x5be0cd19137e2179ull};
    static const uint64_t iv384[8] = {0xcbbb9d5dc1059ed8ull,0x629a292a367cd507ull,0x9159015a3070dd17ull,
        0x152fecd8f70e5939ull,0x67332667ffc00b31ull,0x8eb44a8768581511ull,0xdb0c2e0d64f98fa7ull,
        0x47b5481dbefa4fa4ull};
    memcpy(s->h, is384 ? iv384 : iv512, sizeof iv512); s->nbuf = 0; s->total = 0;
}
static void sha512_update(sha512_t *s, const uint8_t *m, size_t n) {
    s->total += n;
    while (n) {
        size_t k = 128 - s->nbuf; if (k > n) k = n;
        memcpy(s->buf + s->nbuf, m, k); s->nbuf += k; m += k; n -= k;
        if (s->nbuf == 128) { sha512_compress(s->h, s->buf); s->nbuf = 0; }
    }
}
static void sha512_final(sha512_t *s, uint8_t *out, int outlen) {
    uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0, len[16] = {0};
    sha512_update(s, &pad, 1);
    while (s->nbuf != 112) sha512_update(s, &z, 1);
    put_be64(len + 8, bits); sha512_update(s, len, 16);
    uint8_t full[64];
    for (int i = 0; i < 8; i++) put_be64(full + 8 * i, s->h[i]);
    memcpy(out, full, (size_t)outlen);
}
void orc_sha512(const uint8_t *m, size_t n, uint8_t out[64]) {
    sha512_t s; sha512_init_iv(&s, 0); sha512_update(&s, m, n); sha512_final(&s, out, 64);
}
void orc_sha384(const uint8_t *m, size_t n, uint8_t out[48]) {
    sha512_t s; sha512_init_iv(&s, 1); sha512_update(&s, m, n); sha512_final(&s, out, 48);
}

/* ------------------------------------------------------------------ MD5 (RFC 1321) */
typedef struct { uint32_t h[4]; uint8_t buf[64]; size_t nbuf; uint64_t total; } md5_t;
static const uint32_t KMD5[64] = {
    0xd76aa478u,0xe8c7b756u,0x242070dbu,0xc1bdceeeu,0xf57c0fafu,0x4787c62au,0xa8304613u,0xfd469501u,
    0x698098d8u,0x8b44f7afu,0xffff5bb1u,0x895cd7beu,0x6b901122u,0xfd987193u,0xa679438eu,0x49b40821u,
    0xf61e2562u,0xc040b340u,0x265e5a51u,0xe9b6c7aau,0xd62f105du,0x02441453u,0xd8a1e681u,0xe7d3fbc8u,
    0x21e1cde6u,0xc33707d6u,0xf4d50d87u,0x455a14edu,0xa9e3e905u,0xfcefa3f8u,0x676f02d9u,0x8d2a4c8au,
    0xfffa3942u,0x8771f681u,0x6d9d6122u,0xfde5380cu,0xa4beea44u,0x4bdecfa9u,0xf6bb4b60u,0xbebfbc70u,
    0x289b7ec6u,0xeaa127fau,0xd4ef3085u,0x04881d05u,0xd9d4d039u,0xe6db99e5u,0x1fa27cf8u,0xc4ac5665u,
    0xf4292244u,0x432aff97u,0xab9423a7u,0xfc93a039u,0x655b59c3u,0x8f0ccc92u,0xffeff47du,0x85845dd1u,
    0x6fa87e4fu,0xfe2ce6e0u,0xa3014314u,0x4e0811a1u,0xf7537e82u,0xbd3af235u,0x2ad7d2bbu,0xeb86d391u};
static const int SMD5[64] = {7,12,17,22,7,12,17,22,7,12,17,22,7,12,17,22,5,9,14,20,5,9,14,20,5,9,14,20,
    5,9,14,20,4,11,16,23,4,11,16,23,4,11,16,23,4,11,16,23,6,10,15,21,6,10,15,21,6,10,15,21,6,10,15,21};

static void md5_compress(uint32_t h[4], const uint8_t blk[64]) {
    uint32_t m[16];
    CNT(3);
    for (int i = 0; i < 16; i++) m[i] = le32(blk + 4 * i);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f; int g;
        if (i < 16)      { f = (b & c) | (~b & d); g = i; }
        else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
        else if (i < 48) { f = b ^ c ^ d;          g = (3 * i + 5) & 15; }
        else             { f = c ^ (b | ~d);       g = (7 * i) & 15; }
        uint32_t tmp = d; d = c; c = b;
        b = b + rol32(a + f + KMD5[i] + m[g], SMD5[i]);
        a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d;
}
static void md5_init(md5_t *s) {
    s->h[0] = 0x67452301u; s->h[1] = 0xefcdab89u; s->h[2] = 0x98badcfeu; s->h[3] = 0x10325476u;
    s->nbuf = 0; s->total = 0;
}
static void md5_update(md5_t *s, const uint8_t *m, size_t n) {
    s->total += n;
    while (n) {
        size_t k = 64 - s->nbuf; if (k > n) k = n;
        memcpy(s->buf + s->nbuf, m, k); s->nbuf += k; m += k; n -= k;
        if (s->nbuf == 64) { md5_compress(s->h, s->buf); s->nbuf = 0; }
    }
}
static void md5_final(md5_t *s, uint8_t out[16]) {
    uint64_t bits = s->total * 8;
    uint8_t pad = 0x80, z = 0, len[8];
    md5_update(s, &pad, 1);
    while (s->nbuf != 56) md5_update(s, &z, 1);
    put_le32(len, (uint32_t)bits); put_le32(len + 4, (uint32_t)(bits >> 32));
    md5_update(s, len, 8);
    for (int i = 0; i < 4; i++) put_le32(out + 4 * i, s->h[i]);
}
void orc_md5(const uint8_t *m, size_t n, uint8_t out[16]) {
    md5_t s; md5_init(&s); md5_update(&s, m, n); md5_final(&s, out);
}

/* ------------------------------------------------------------------ AES (FIPS 197), byte oriented */
static uint8_t SBOX[256], INV_SBOX[256];
static pthread_once_t aes_once = PTHREAD_ONCE_INIT;

static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}
static void aes_tables_init(void) {
    /* S-box = affine transform of the multiplicative inverse in GF(2^8) (FIPS 197 5.1.1) */
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) for (int y = 1; y < 256; y++) if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
        s ^= 0x63;
        SBOX[x] = s; INV_SBOX[s] = (uint8_t)x;
    }
}
static int aes_expand(const uint8_t *key, int keybits, uint8_t rk[240]) {
    pthread_once(&aes_once, aes_tables_init);
    int nk = keybits / 32, nr = nk + 6;
    CNT(keybits == 128 ? 8 : 9);
    memcpy(rk, key, (size_t)(4 * nk));
    uint8_t rcon = 1;
    for (int i = nk; i < 4 * (nr + 1); i++) {
        uint8_t t[4]; memcpy(t, rk + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rcon); t[1] = SBOX[t[2]]; t[2] = SBOX[t[3]]; t[3] = SBOX[u];
            rcon = (uint8_t)((rcon << 1) ^ ((rcon & 0x80) ? 0x1b : 0));
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; j++) t[j] = SBOX[t[j]];
        }
        for (int j = 0; j < 4; j++) rk[4 * i + j] = (uint8_t)(rk[4 * (i - nk) + j] ^ t[j]);
    }
    return nr;
}
static void aes_enc_rk(const uint8_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int r = 1; r <= nr; r++) {
        for (int i = 0; i < 16; i++) t[i] = SBOX[s[(i + 4 * (i % 4)) % 16]];  /* SubBytes+ShiftRows */
        if (r != nr) {
            for (int c = 0; c < 4; c++) {
                uint8_t *p = t + 4 * c, a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
                p[0] = gmul(a0, 2) ^ gmul(a1, 3) ^ a2 ^ a3;
                p[1] = a0 ^ gmul(a1, 2) ^ gmul(a2, 3) ^ a3;
                p[2] = a0 ^ a1 ^ gmul(a2, 2) ^ gmul(a3, 3);
                p[3] = gmul(a0, 3) ^ a1 ^ a2 ^ gmul(a3, 2);
            }
        }
        for (int i = 0; i < 16; i++) s[i] = t[i] ^ rk[16 * r + i];
    }
    memcpy(out, s, 16);
}
static void aes_dec_rk(const uint8_t *rk, int nr, const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16], t[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[16 * nr + i];
    for (int r = nr - 1; r >= 0; r--) {
        for (int i = 0; i < 16; i++) t[(i + 4 * (i % 4)) % 16] = INV_SBOX[s[i]];  /* InvShiftRows+InvSubBytes */
        for (int i = 0; i < 16; i++) t[i] ^= rk[16 * r + i];
        if (r != 0) {
            for (int c = 0; c < 4; c++) {
                uint8_t *p = t + 4 * c, a0 = p[0], a1 = p[1], a2 = p[2], a3 = p[3];
                p[0] = gmul(a0, 14) ^ gmul(a1, 11) ^ gmul(a2, 13) ^ gmul(a3, 9);
                p[1] = gmul(a0, 9) ^ gmul(a1, 14) ^ gmul(a2, 11) ^ gmul(a3, 13);
                p[2] = gmul(a0, 13) ^ gmul(a1, 9) ^ gmul(a2, 14) ^ gmul(a3, 11);
                p[3] = gmul(a0, 11) ^ gmul(a1, 13) ^ gmul(a2, 9) ^ gmul(a3, 14);
            }
        }
        memcpy(s, t, 16);
    }
    memcpy(out, s, 16);
}
void orc_aes_encrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240]; int nr = aes_expand(key, keybits, rk); aes_enc_rk(rk, nr, in, out);
}
void orc_aes_decrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[240]; int nr = aes_expand(key, keybits, rk); aes_dec_rk(rk, nr, in, out);
}

/* ------------------------------------------------------------------ RC4 */
void orc_rc4(const uint8_t *key, int keylen, const uint8_t *in, size_t n, uint8_t *out) {
    uint8_t S[256]; int i, j = 0;
    CNT(6);
    for (i = 0; i < 256; i++) S[i] = (uint8_t)i;
    for (i = 0; i < 256; i++) {
        j = (j + S[i] + key[i % keylen]) & 255;
        uint8_t t = S[i]; S[i] = S[j]; S[j] = t;
    }
    i = 0; j = 0;
    for (size_t k = 0; k < n; k++) {
        CNT(7);
        i = (i + 1) & 255; j = (j + S[i]) & 255;
        uint8_t t = S[i]; S[i] = S[j]; S[j] = t;
        out[k] = in[k] ^ S[(S[i] + S[j]) & 255];
    }
}

/* ------------------------------------------------------------------ PBKDF2-HMAC-SHA1 (RFC 8018 5.2)
 * HMAC keyed once: the ipad/opad blocks are absorbed into two saved SHA-1 states (as OpenSSL's HMAC_CTX
 * does), so each iteration costs exactly two compressions. */
typedef struct { sha1_t in, out; } hmac_sha1_t;
static void hmac_sha1_key(hmac_sha1_t *h, const uint8_t *key, size_t klen) {
    uint8_t k0[64] = {0}, ip[64], op[64];
    if (klen > 64) orc_sha1(key, klen, k0); else memcpy(k0, key, klen);
    for (int i = 0; i < 64; i++) { ip[i] = k0[i] ^ 0x36; op[i] = k0[i] ^ 0x5c; }
    sha1_init(&h->in); sha1_update(&h->in, ip, 64);
    sha1_init(&h->out); sha1_update(&h->out, op, 64);
}
static void hmac_sha1_run(const hmac_sha1_t *h, const uint8_t *m, size_t n, uint8_t out[20]) {
    uint8_t inner[20];
    sha1_t s = h->in; sha1_update(&s, m, n); sha1_final(&s, inner);
    s = h->out; sha1_update(&s, inner, 20); sha1_final(&s, out);
}
void orc_pbkdf2_hmac_sha1(const uint8_t *pw, size_t pwlen, const uint8_t *salt, size_t saltlen,
                          uint32_t iters, uint8_t *out, size_t outlen) {
    hmac_sha1_t h;
    hmac_sha1_key(&h, pw, pwlen);
    uint8_t *msg = (uint8_t *)malloc(saltlen + 4);
    memcpy(msg, salt, saltlen);
    for (uint32_t blk = 1; outlen; blk++) {
        uint8_t u[20], t[20];
        put_be32(msg + saltlen, blk);
        hmac_sha1_run(&h, msg, saltlen + 4, u);
        memcpy(t, u, 20);
        for (uint32_t it = 1; it < iters; it++) {
            hmac_sha1_run(&h, u, 20, u);
            for (int k = 0; k < 20; k++) t[k] ^= u[k];
        }
        size_t k = outlen < 20 ? outlen : 20;
        memcpy(out, t, k); out += k; outlen -= k;
    }
    free(msg);
}

/* ------------------------------------------------------------------ str_to_uchar (BN_hex2bn + BN_bn2bin) */
static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
int orc_bn_hex_decode(const char *hex, uint8_t *out, int cap) {
    /* BN_hex2bn: optional '-', then the longest run of hex digits; BN_bn2bin writes the magnitude
     * big-endian in BN_num_bytes bytes, i.e. WITHOUT leading zero bytes (msoffcrypto...c:340-349). */
    if (*hex == '-') hex++;
    int nd = 0;
    while (hexval((unsigned char)hex[nd]) >= 0) nd++;
    int skip = 0;
    while (skip < nd && hexval((unsigned char)hex[skip]) == 0) skip++;  /* leading zero digits */
    int sig = nd - skip;                  /* significant digits */
    int nbytes = (sig + 1) / 2;
    if (nbytes > cap) return nbytes;      /* caller treats as overflow */
    /* right-align digits into nbytes, big-endian */
    for (int b = 0; b < nbytes; b++) {
        int lo_idx = nd - 1 - 2 * (nbytes - 1 - b);   /* index of low nibble digit */
        int hi_idx = lo_idx - 1;
        int lo = hexval((unsigned char)hex[lo_idx]);
        int hi = (hi_idx >= skip) ? hexval((unsigned char)hex[hi_idx]) : 0;
        out[b] = (uint8_t)((hi << 4) | lo);
    }
    return nbytes;
}

/* ------------------------------------------------------------------ contexts */
struct orc_ctx {
    int fmt, flags;
    /* office */
    uint8_t salt[64]; int salt_len; uint8_t ev[128]; int ev_len; uint8_t evh[128]; int evh_len;
    int key_bits, hash_size;
    /* odt */
    uint8_t checksum[32], iv[16], osalt[16]; uint8_t *enc; int enc_len;
    /* pdf */
    int V, R, Length, P, meta; uint8_t id[256]; int id_len; uint8_t u[256]; int u_len;
    uint8_t o[256]; int o_len;
};

/* Decode a hex field into a buffer of the length the reference declares (its VLA); tail bytes the
 * reference leaves uninitialised are zeroed here and the ctx is flagged.  Returns <0 on overflow. */
static int decode_field(orc_ctx *c, const char *hex, uint8_t *buf, int declared) {
    memset(buf, 0, (size_t)(declared > 0 ? declared : 0));
    if (declared <= 0) return 0;
    int n = orc_bn_hex_decode(hex, buf, declared);
    if (n > declared) return -1;
    if (n < declared) c->flags |= ORC_FLAG_REF_NONDETERMINISTIC;
    return 0;
}

static int py2_half_len(const char *s) { return (int)(strlen(s) / 2); }   /* len(x) / 2 in Python 2 */

int orc_ctx_create(const char *const *fields, int nfields, orc_ctx **out) {
    *out = NULL;
    if (nfields < 1) return -1;
    orc_ctx *c = (orc_ctx *)calloc(1, sizeof *c);
    const char *tag = fields[0];
    if (!strcmp(tag, "office") && nfields == 8) {
        /* argv mapping brute_force.py:163-173 */
        c->fmt = ORC_FMT_OFFICE;
        c->salt_len = atoi(fields[4]);
        c->ev_len = py2_half_len(fields[6]);
        c->evh_len = py2_half_len(fields[7]);
        c->key_bits = atoi(fields[3]);
        c->hash_size = atoi(fields[2]);
        if (c->salt_len < 16 || c->salt_len > 64 || c->ev_len > 128 || c->evh_len > 128) goto bad;
        if (c->ev_len % 16 || c->evh_len % 16) goto bad;       /* EVP_DecryptFinal_ex -> abort() */
        if (c->key_bits < 128) goto bad;                        /* finalKey shorter than AES-128 reads */
        if (decode_field(c, fields[5], c->salt, c->salt_len) < 0) goto bad;
        if (decode_field(c, fields[6], c->ev, c->ev_len) < 0) goto bad;
        if (decode_field(c, fields[7], c->evh, c->evh_len) < 0) goto bad;
        if (c->ev_len != 16 || c->evh_len != 32) c->flags |= ORC_FLAG_NEVER_MATCHES; /* :163, :168 */
        else if (c->hash_size < 0 || c->hash_size >= 32) goto bad; /* reads uninitialised plaintext */
    } else if (!strcmp(tag, "odt") && nfields == 7) {
        /* argv mapping brute_force.py:175-182 */
        c->fmt = ORC_FMT_ODT;
        c->enc_len = atoi(fields[6]);
        if (c->enc_len < 0 || c->enc_len % 16) goto bad;       /* EVP_DecryptFinal_ex -> abort() */
        c->enc = (uint8_t *)calloc((size_t)c->enc_len + 16, 1);
        if (decode_field(c, fields[2], c->checksum, 32) < 0) goto bad;
        if (decode_field(c, fields[3], c->iv, 16) < 0) goto bad;
        if (decode_field(c, fields[4], c->osalt, 16) < 0) goto bad;
        if (decode_field(c, fields[5], c->enc, c->enc_len) < 0) goto bad;
    } else if (!strcmp(tag, "pdf") && nfields == 12) {
        /* argv mapping brute_force.py:184-197 */
        c->fmt = ORC_FMT_PDF;
        c->V = atoi(fields[1]); c->R = atoi(fields[2]); c->Length = atoi(fields[3]);
        c->P = atoi(fields[4]); c->meta = atoi(fields[5]);
        c->id_len = atoi(fields[6]); c->u_len = atoi(fields[8]); c->o_len = atoi(fields[10]);
        if (c->id_len < 0 || c->id_len > 256 || c->u_len < 0 || c->u_len > 256 || c->o_len < 0 || c->o_len > 256)
            goto bad;
        if (decode_field(c, fields[7], c->id, c->id_len) < 0) goto bad;
        if (decode_field(c, fields[9], c->u, c->u_len) < 0) goto bad;
        if (decode_field(c, fields[11], c->o, c->o_len) < 0) goto bad;
        int V = c->V, R = c->R;
        /* (V,R) whitelist and Length % 8 (pdf...c:89-101) */
        if ((V != 1 && V != 2 && V != 4 && V != 5) || (V == 1 && R != 2) || (V == 2 && R != 3) ||
            (V == 4 && R != 4) || (V == 5 && (R != 5 && R != 6)) || (c->Length % 8 != 0)) {
            c->flags |= ORC_FLAG_NEVER_MATCHES;
        } else if (R >= 5) {
            if (c->u_len < 40) goto bad;                        /* reads u[32..40) */
        } else {
            int n = c->Length / 8;
            if (R == 2 && (n < 5 || c->u_len < 32)) goto bad;   /* rc4_40 key = hash[0:5] */
            if (R >= 3 && ((n != 5 && n != 16) || c->u_len < 16)) goto bad; /* EVP_rc4 reads 16 B of key */
        }
    } else {
        goto bad;
    }
    *out = c;
    return 0;
bad:
    free(c->enc);
    free(c);
    return -1;
}
void orc_ctx_destroy(orc_ctx *c) { if (c) { free(c->enc); free(c); } }
int orc_ctx_format(const orc_ctx *c) { return c->fmt; }
int orc_ctx_flags(const orc_ctx *c) { return c->flags; }

/* UTF-8 -> UTF-16LE as glibc iconv("UTF16LE","UTF8") does for valid input (msoffcrypto...c:275-336). */
static int utf8_to_utf16le(const uint8_t *s, int n, uint8_t *out, int cap) {
    int o = 0;
    for (int i = 0; i < n;) {
        uint32_t cp; int k;
        uint8_t b = s[i];
        if (b < 0x80) { cp = b; k = 1; }
        else if ((b & 0xE0) == 0xC0) { cp = b & 0x1F; k = 2; }
        else if ((b & 0xF0) == 0xE0) { cp = b & 0x0F; k = 3; }
        else if ((b & 0xF8) == 0xF0) { cp = b & 0x07; k = 4; }
        else return -1;
        if (i + k > n) return -1;
        for (int j = 1; j < k; j++) {
            if ((s[i + j] & 0xC0) != 0x80) return -1;
            cp = (cp << 6) | (s[i + j] & 0x3F);
        }
        if ((k == 2 && cp < 0x80) || (k == 3 && cp < 0x800) || (k == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
            return -1;
        if (cp >= 0xD800 && cp <= 0xDFFF) return -1;
        if (cp >= 0x10000) {
            if (o + 4 > cap) return -1;
            uint32_t v = cp - 0x10000, hi = 0xD800 | (v >> 10), lo = 0xDC00 | (v & 0x3FF);
            out[o++] = (uint8_t)hi; out[o++] = (uint8_t)(hi >> 8); out[o++] = (uint8_t)lo; out[o++] = (uint8_t)(lo >> 8);
        } else {
            if (o + 2 > cap) return -1;
            out[o++] = (uint8_t)cp; out[o++] = (uint8_t)(cp >> 8);
        }
        i += k;
    }
    return o;
}

/* Office: verify() msoffcrypto_password_verifier.c:56-191.  inter (may be NULL) receives
 * finalH[20] | X1[20] | key[16] | sha1(verifier)[20] | dec_evh[0:20] */
static int verify_office(const orc_ctx *c, const uint8_t *pw, int len, uint8_t *inter) {
    if (len <= 0) return -1;                 /* iconv of "" -> -1, then uninitialised length (:287-292) */
    /* any length (iconv's buffer grows, :306-323): 2 bytes of UTF-16LE per UTF-8 byte at most */
    uint8_t *u16 = (uint8_t *)malloc((size_t)len * 2);
    int ulen = utf8_to_utf16le(pw, len, u16, len * 2);
    if (ulen < 0) { free(u16); return -1; }  /* iconv failure: reference continues on freed memory */
    /* H0 = SHA1(salt[0:16] || pwU16) over salt_len + ulen bytes, zero tail (:94-101) */
    size_t mlen = (size_t)c->salt_len + (size_t)ulen;
    uint8_t *msg = (uint8_t *)calloc(mlen, 1);
    memcpy(msg, c->salt, 16);
    memcpy(msg + 16, u16, (size_t)ulen);
    free(u16);
    uint8_t h[20], tmp[24];
    orc_sha1(msg, mlen, h);
    free(msg);
    /* 50,000 x H = SHA1(LE32(i) || H) (:105-113) */
    for (uint32_t i = 0; i < 50000; i++) {
        put_le32(tmp, i); memcpy(tmp + 4, h, 20);
        orc_sha1(tmp, 24, h);
    }
    /* H = SHA1(H || 00000000) (:115-118) */
    memcpy(tmp, h, 20); memset(tmp + 20, 0, 4);
    orc_sha1(tmp, 24, h);
    /* X1 = SHA1((0x36 x 64) ^ H), key = X1[0:16] -- AES-128-ECB always (:128-153, :207) */
    uint8_t x1in[64], x1[20];
    memset(x1in, 0x36, 64);
    for (int x = 0; x < 20; x++) x1in[x] ^= h[x];
    orc_sha1(x1in, 64, x1);
    if (inter) { memcpy(inter, h, 20); memcpy(inter + 20, x1, 20); memcpy(inter + 40, x1, 16); }
    if (c->flags & ORC_FLAG_NEVER_MATCHES) return 0;
    uint8_t rk[240], dv[16], dh[32], vh[20];
    int nr = aes_expand(x1, 128, rk);
    aes_dec_rk(rk, nr, c->ev, dv);
    aes_dec_rk(rk, nr, c->evh, dh);
    aes_dec_rk(rk, nr, c->evh + 16, dh + 16);
    if (dh[c->hash_size] != 0x00) return 0;  /* (:168) */
    orc_sha1(dv, 16, vh);                    /* (:175) */
    if (inter) { memcpy(inter + 56, vh, 20); memcpy(inter + 76, dh, 20); }
    return memcmp(vh, dh, 20) == 0;          /* (:184-188) */
}

/* ODT: verify() odt_password_verifier.c:51-126.  inter: start_key[32] | derived_key[32] | hash[32] */
static int verify_odt(const orc_ctx *c, const uint8_t *pw, int len, uint8_t *inter) {
    uint8_t sk[32], dk[32];
    orc_sha256(pw, (size_t)len, sk);                                 /* (:78-79) */
    orc_pbkdf2_hmac_sha1(sk, 32, c->osalt, 16, 1024, dk, 32);       /* (:85) iteration count fixed */
    if (inter) { memcpy(inter, sk, 32); memcpy(inter + 32, dk, 32); }
    /* AES-256-CBC decrypt, no padding (:90-92, :133-161) */
    uint8_t rk[240];
    int nr = aes_expand(dk, 256, rk);
    if (c->enc_len == 16) {                                          /* (:98-101) */
        uint8_t p[16];
        aes_dec_rk(rk, nr, c->enc, p);
        CNT(5);
        for (int k = 0; k < 16; k++) p[k] ^= c->iv[k];
        return p[0] == 0x03 && p[1] == 0x00;
    }
    int n = c->enc_len > 1024 ? 1024 : c->enc_len;                   /* (:104-106) */
    uint8_t *p = (uint8_t *)malloc((size_t)n + 16);
    const uint8_t *prev = c->iv;
    for (int b = 0; b < n / 16; b++) {
        aes_dec_rk(rk, nr, c->enc + 16 * b, p + 16 * b);
        CNT(5);
        for (int k = 0; k < 16; k++) p[16 * b + k] ^= prev[k];
        prev = c->enc + 16 * b;
    }
    uint8_t hh[32];
    orc_sha256(p, (size_t)n, hh);                                    /* (:111) */
    free(p);
    if (inter) memcpy(inter + 64, hh, 32);
    return memcmp(hh, c->checksum, 32) == 0;                         /* (:119-123) */
}

static const uint8_t PDF_PAD[32] = {0x28,0xBF,0x4E,0x5E,0x4E,0x75,0x8A,0x41,0x64,0x00,0x4E,0x56,0xFF,0xFA,
    0x01,0x08,0x2E,0x2E,0x00,0xB6,0xD0,0x68,0x3E,0x80,0x2F,0x0C,0xA9,0xFE,0x64,0x53,0x69,0x7A};

/* pdf_compute_hardened_hash_r6 (pdf...c:226-291), ownerkey == NULL */
static void pdf_r6_hash(const uint8_t *pw, int pwlen, const uint8_t salt[8], uint8_t out[32]) {
    uint8_t block[64];
    int bs = 32;
    sha256_t s;
    sha256_init(&s); sha256_update(&s, pw, (size_t)pwlen); sha256_update(&s, salt, 8); sha256_final(&s, block);
    size_t dlen = 0;
    uint8_t *data = (uint8_t *)malloc((size_t)(pwlen + 64) * 64);
    uint8_t last = 0;
    for (int i = 0; i < 64 || i < (int)last + 32; i++) {              /* (:247) */
        dlen = (size_t)(pwlen + bs);
        for (int j = 0; j < 64; j++) {                                   /* (:250-256) */
            memcpy(data + j * dlen, pw, (size_t)pwlen);
            memcpy(data + j * dlen + pwlen, block, (size_t)bs);
        }
        uint8_t rk[240], chain[16];
        int nr = aes_expand(block, 128, rk);                             /* (:259) */
        memcpy(chain, block + 16, 16);
        for (size_t b = 0; b < dlen * 64 / 16; b++) {                   /* (:261) CBC encrypt */
            uint8_t x[16];
            for (int k = 0; k < 16; k++) x[k] = data[16 * b + k] ^ chain[k];
            aes_enc_rk(rk, nr, x, data + 16 * b);
            CNT(4);
            memcpy(chain, data + 16 * b, 16);
        }
        int sum = 0;
        for (int j = 0; j < 16; j++) sum += data[j];                     /* (:264-265) */
        bs = 32 + (sum % 3) * 16;                                        /* (:268) */
        if (bs == 32) orc_sha256(data, dlen * 64, block);
        else if (bs == 48) orc_sha384(data, dlen * 64, block);
        else orc_sha512(data, dlen * 64, block);
        last = data[dlen * 64 - 1];
    }
    free(data);
    memcpy(out, block, 32);
}

/* PDF: verify() pdf_password_verifier.c:64-192.  inter: R<=4 padded[32] | initial hash[16] | U'[32];
 * R5/R6: computed hash[32] */
static int verify_pdf(const orc_ctx *c, const uint8_t *pw, int len, uint8_t *inter) {
    if (c->flags & ORC_FLAG_NEVER_MATCHES) return 0;
    int R = c->R;
    if (R == 5) {                                                        /* verify_user_r5 :194-221 */
        uint8_t buf[136], hh[32];
        int pl = len > 127 ? 127 : len;
        memcpy(buf, pw, (size_t)pl); memcpy(buf + pl, c->u + 32, 8);
        orc_sha256(buf, (size_t)pl + 8, hh);
        if (inter) memcpy(inter, hh, 32);
        return memcmp(hh, c->u, 32) == 0;
    }
    if (R == 6) {                                                        /* :115-132 */
        /* data[(128 + 64 + 48) * 64] (:228) holds 64 x (pw || K[0:64]) up to pwlen 176; longer passwords overflow it
         * and the reference aborts (stack protector, measured: tests/golden/long_verdicts.json) */
        if (len > 176) return -1;
        uint8_t hh[32];
        pdf_r6_hash(pw, len, c->u + 32, hh);
        if (inter) memcpy(inter, hh, 32);
        return memcmp(hh, c->u, 32) == 0;
    }
    /* Algorithm 2 (:136-158) */
    uint8_t pass[32], hash[16];
    int pl = len <= 32 ? len : 32;
    memcpy(pass, pw, (size_t)pl); memcpy(pass + pl, PDF_PAD, (size_t)(32 - pl));
    md5_t m;
    md5_init(&m);
    md5_update(&m, pass, 32);
    md5_update(&m, c->o, (size_t)c->o_len);
    uint8_t pb[4]; put_le32(pb, (uint32_t)c->P); md5_update(&m, pb, 4);
    md5_update(&m, c->id, (size_t)c->id_len);
    if (R >= 4 && !c->meta) { static const uint8_t ff[4] = {0xff, 0xff, 0xff, 0xff}; md5_update(&m, ff, 4); }
    md5_final(&m, hash);
    int n = c->Length / 8;
    if (inter) { memcpy(inter, pass, 32); memcpy(inter + 32, hash, 16); }
    if (R >= 3) for (int i = 0; i < 50; i++) orc_md5(hash, (size_t)n, hash);   /* (:150-155) */
    uint8_t key[16];
    memcpy(key, hash, (size_t)(n < 16 ? n : 16));
    uint8_t ct[32] = {0};
    if (R == 2) {
        orc_rc4(key, 5, PDF_PAD, 32, ct);                                /* (:161-163) rc4_40 */
    } else {
        uint8_t h2[16], x[16];
        md5_init(&m); md5_update(&m, PDF_PAD, 32); md5_update(&m, c->id, (size_t)c->id_len); md5_final(&m, h2);
        orc_rc4(key, n, h2, 16, ct);                                     /* (:167-168) */
        for (int r = 1; r <= 19; r++) {                                  /* (:170-174) */
            for (int i = 0; i < n; i++) x[i] = key[i] ^ (uint8_t)r;
            orc_rc4(x, n, ct, 16, ct);
        }
        memcpy(ct + 16, PDF_PAD, 16);
    }
    if (inter) memcpy(inter + 48, ct, 32);
    int boundary = R >= 3 ? 16 : 32;                                     /* (:184-189) */
    return memcmp(c->u, ct, (size_t)boundary) == 0;
}

static int verify_any(const orc_ctx *c, const uint8_t *pw, int len, uint8_t *inter) {
    switch (c->fmt) {
        case ORC_FMT_OFFICE: return verify_office(c, pw, len, inter);
        case ORC_FMT_ODT: return verify_odt(c, pw, len, inter);
        case ORC_FMT_PDF: return verify_pdf(c, pw, len, inter);
    }
    return -1;
}
int orc_verify(const orc_ctx *c, const uint8_t *pw, int len) { return verify_any(c, pw, len, NULL); }

int orc_intermediates(const orc_ctx *c, const uint8_t *pw, int len, uint8_t *out, int cap) {
    uint8_t buf[128] = {0};
    int r = verify_any(c, pw, len, buf);
    if (r < 0) return r;
    int n = cap < 128 ? cap : 128;
    memcpy(out, buf, (size_t)n);
    return n;
}

int orc_work_counts(const orc_ctx *c, const uint8_t *pw, int len, uint64_t counts[ORC_NCOUNT]) {
    memset(g_cnt, 0, sizeof g_cnt);
    int r = verify_any(c, pw, len, NULL);
    memcpy(counts, g_cnt, sizeof g_cnt);
    return r;
}

/* ------------------------------------------------------------------ enumeration + threaded search */
/* index -> password in itertools.product(charset, repeat=pwlen) order (brute_force.py:205):
 * the leftmost character is the most significant digit. */
static void index_to_pw(uint64_t idx, const uint8_t *cs, int cslen, int pwlen, uint8_t *pw) {
    for (int p = pwlen - 1; p >= 0; p--) { pw[p] = cs[idx % (uint64_t)cslen]; idx /= (uint64_t)cslen; }
}

typedef struct {
    const orc_ctx *c; const uint8_t *cs; int cslen, pwlen; uint64_t start, count;
    uint64_t *hits; int64_t cap, nhits; int err;
    /* list mode */
    const uint8_t *blob; const uint64_t *offs; int8_t *verdicts;
} job_t;

static void *range_worker(void *arg) {
    job_t *j = (job_t *)arg;
    uint8_t pw[256];
    for (uint64_t k = 0; k < j->count; k++) {
        uint64_t idx = j->start + k;
        index_to_pw(idx, j->cs, j->cslen, j->pwlen, pw);
        int r = orc_verify(j->c, pw, j->pwlen);
        if (r < 0) { j->err = r; return NULL; }
        if (r) { if (j->nhits < j->cap) j->hits[j->nhits] = idx; j->nhits++; }
    }
    return NULL;
}

int64_t orc_search_range(const orc_ctx *c, const uint8_t *cs, int cslen, int pwlen, uint64_t start,
                         uint64_t count, int nthreads, uint64_t *hits, int64_t cap) {
    if (nthreads < 1) nthreads = 1;
    if (pwlen < 1 || pwlen > 255 || cslen < 1) return -1;
    if ((uint64_t)nthreads > count) nthreads = count ? (int)count : 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t per = count / (uint64_t)nthreads, rem = count % (uint64_t)nthreads, s = start;
    for (int t = 0; t < nthreads; t++) {
        job_t *j = &jobs[t];
        j->c = c; j->cs = cs; j->cslen = cslen; j->pwlen = pwlen;
        j->start = s; j->count = per + ((uint64_t)t < rem ? 1 : 0); s += j->count;
        j->cap = cap; j->hits = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(cap > 0 ? cap : 1));
        pthread_create(&th[t], NULL, range_worker, j);
    }
    int64_t total = 0; int err = 0;
    for (int t = 0; t < nthreads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].err) err = jobs[t].err;
        for (int64_t k = 0; k < jobs[t].nhits && k < jobs[t].cap; k++)
            if (total + k < cap) hits[total + k] = jobs[t].hits[k];
        total += jobs[t].nhits;
        free(jobs[t].hits);
    }
    free(jobs); free(th);
    return err ? err : total;
}

static void *list_worker(void *arg) {
    job_t *j = (job_t *)arg;
    for (uint64_t k = j->start; k < j->start + j->count; k++) {
        int r = orc_verify(j->c, j->blob + j->offs[k], (int)(j->offs[k + 1] - j->offs[k]));
        j->verdicts[k] = (int8_t)r;
    }
    return NULL;
}

int orc_verify_list(const orc_ctx *c, const uint8_t *blob, const uint64_t *offsets, int64_t n,
                    int nthreads, int8_t *verdicts) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n) nthreads = n > 0 ? (int)n : 1;
    job_t *jobs = (job_t *)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    uint64_t per = (uint64_t)n / (uint64_t)nthreads, rem = (uint64_t)n % (uint64_t)nthreads, s = 0;
    for (int t = 0; t < nthreads; t++) {
        job_t *j = &jobs[t];
        j->c = c; j->blob = blob; j->offs = offsets; j->verdicts = verdicts;
        j->start = s; j->count = per + ((uint64_t)t < rem ? 1 : 0); s += j->count;
        pthread_create(&th[t], NULL, list_worker, j);
    }
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(jobs); free(th);
    return 0;
}

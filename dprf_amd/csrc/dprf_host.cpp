/* dprf_host.cpp -- the C ABI of libdprf.so (include/dprf.h): per-document contexts, keyspace and list
 * batching, launches on the context's HIP stream, hit collection and timing.
 *
 * Replaces, per candidate batch, what brute_force.py does per candidate: the argv mapping
 * (_call_*_core, brute_force.py:163-197) becomes one context created from the field array; the
 * JoinableQueue + Popen + wait() loop (:106-161) becomes chunked kernel launches, and the 4 worker
 * processes on one queue (:70-73, :92-95) become one worker thread + HIP stream per GPU of the context on
 * one shared chunk cursor.  No verification
 * runs on the host: a context whose reference verdict is constant (DPRF_FLAG_NEVER_MATCHES) is the
 * only case that launches nothing.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dprf.h"
#include "dprf_launch.h"
#include "dprf_params.h"

/* ------------------------------------------------------------------ errors */
static thread_local std::string g_err;
static int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(DPRF_E_HIP, "%s: %s", #x, hipGetErrorString(e_));  \
    } while (0)

/* ------------------------------------------------------------------ AES tables (FIPS 197 5.1.1) */
static uint8_t gmul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    while (b) {
        if (b & 1) p ^= a;
        a = (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0));
        b >>= 1;
    }
    return p;
}
static dprf_aes_tables make_tables() {
    dprf_aes_tables t;
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x)
            for (int y = 1; y < 256; y++)
                if (gmul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        uint8_t s = inv, r = inv;
        for (int i = 0; i < 4; i++) { r = (uint8_t)((r << 1) | (r >> 7)); s ^= r; }
        s ^= 0x63;
        t.sbox[x] = s;
        t.inv_sbox[s] = (uint8_t)x;
    }
    for (int x = 0; x < 256; x++) {
        uint8_t s = t.sbox[x], i = t.inv_sbox[x];
        t.te0[x] = ((uint32_t)gmul(s, 2) << 24) | ((uint32_t)s << 16) | ((uint32_t)s << 8) | gmul(s, 3);
        t.td0[x] = ((uint32_t)gmul(i, 14) << 24) | ((uint32_t)gmul(i, 9) << 16) | ((uint32_t)gmul(i, 13) << 8) |
                   gmul(i, 11);
    }
    return t;
}
static const dprf_aes_tables &aes_tables() {
    static const dprf_aes_tables t = make_tables();
    return t;
}

/* ------------------------------------------------------------------ host MD5 (RFC 1321), for the
 * document constant MD5(PAD || ID) only */
static void md5_host(const uint8_t *msg, size_t n, uint8_t out[16]) {
    static const uint32_t K[64] = {
        0xd76aa478u,0xe8c7b756u,0x242070dbu,0xc1bdceeeu,0xf57c0fafu,0x4787c62au,0xa8304613u,0xfd469501u,
        0x698098d8u,0x8b44f7afu,0xffff5bb1u,0x895cd7beu,0x6b901122u,0xfd987193u,0xa679438eu,0x49b40821u,
        0xf61e2562u,0xc040b340u,0x265e5a51u,0xe9b6c7aau,0xd62f105du,0x02441453u,0xd8a1e681u,0xe7d3fbc8u,
        0x21e1cde6u,0xc33707d6u,0xf4d50d87u,0x455a14edu,0xa9e3e905u,0xfcefa3f8u,0x676f02d9u,0x8d2a4c8au,
        0xfffa3942u,0x8771f681u,0x6d9d6122u,0xfde5380cu,0xa4beea44u,0x4bdecfa9u,0xf6bb4b60u,0xbebfbc70u,
        0x289b7ec6u,0xeaa127fau,0xd4ef3085u,0x04881d05u,0xd9d4d039u,0xe6db99e5u,0x1fa27cf8u,0xc4ac5665u,
        0xf4292244u,0x432aff97u,0xab9423a7u,0xfc93a039u,0x655b59c3u,0x8f0ccc92u,0xffeff47du,0x85845dd1u,
        0x6fa87e4fu,0xfe2ce6e0u,0xa3014314u,0x4e0811a1u,0xf7537e82u,0xbd3af235u,0x2ad7d2bbu,0xeb86d391u};
    static const int S[16] = {7, 12, 17, 22, 5, 9, 14, 20, 4, 11, 16, 23, 6, 10, 15, 21};
    std::vector<uint8_t> m(msg, msg + n);
    m.push_back(0x80);
    while (m.size() % 64 != 56) m.push_back(0);
    uint64_t bits = (uint64_t)n * 8;
    for (int i = 0; i < 8; i++) m.push_back((uint8_t)(bits >> (8 * i)));
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    for (size_t off = 0; off < m.size(); off += 64) {
        uint32_t w[16];
        for (int i = 0; i < 16; i++)
            w[i] = (uint32_t)m[off + 4 * i] | ((uint32_t)m[off + 4 * i + 1] << 8) |
                   ((uint32_t)m[off + 4 * i + 2] << 16) | ((uint32_t)m[off + 4 * i + 3] << 24);
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
        for (int i = 0; i < 64; i++) {
            uint32_t f;
            int g;
            if (i < 16) { f = (b & c) | (~b & d); g = i; }
            else if (i < 32) { f = (d & b) | (~d & c); g = (5 * i + 1) & 15; }
            else if (i < 48) { f = b ^ c ^ d; g = (3 * i + 5) & 15; }
            else { f = c ^ (b | ~d); g = (7 * i) & 15; }
            uint32_t tmp = d;
            d = c;
            c = b;
            uint32_t x = a + f + K[i] + w[g];
            int s = S[(i >> 4) * 4 + (i & 3)];
            b = b + ((x << s) | (x >> (32 - s)));
            a = tmp;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d;
    }
    for (int i = 0; i < 4; i++)
        for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
}

/* ------------------------------------------------------------------ field decoding */
static int hexval(int c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}
/* The reference decodes with str_to_uchar (BN_hex2bn + BN_bn2bin, msoffcrypto...c:340-349) into a
 * buffer of the length its argv declares.  Inside the parity domain the string is exactly 2*declared
 * hex digits; a leading 00 byte makes the reference decode short (flagged, decoded in full here). */
static int decode_hex(const char *s, int declared, std::vector<uint8_t> &out, int &flags, const char *what) {
    size_t n = strlen(s);
    if (declared < 0 || n != (size_t)declared * 2)
        return fail(DPRF_E_DOMAIN, "%s: %zu hex digits for a declared length of %d bytes", what, n, declared);
    out.resize((size_t)declared);
    for (int i = 0; i < declared; i++) {
        int hi = hexval((unsigned char)s[2 * i]), lo = hexval((unsigned char)s[2 * i + 1]);
        if (hi < 0 || lo < 0) return fail(DPRF_E_DOMAIN, "%s: not a hex string", what);
        out[i] = (uint8_t)(hi << 4 | lo);
    }
    if (declared > 0 && out[0] == 0) flags |= DPRF_FLAG_REF_NONDETERMINISTIC;
    return DPRF_OK;
}
static uint32_t be_word(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static uint32_t le_word(const uint8_t *p) {
    return ((uint32_t)p[3] << 24) | ((uint32_t)p[2] << 16) | ((uint32_t)p[1] << 8) | p[0];
}
static const uint8_t PDF_PAD[32] = {0x28, 0xBF, 0x4E, 0x5E, 0x4E, 0x75, 0x8A, 0x41, 0x64, 0x00, 0x4E,
                                    0x56, 0xFF, 0xFA, 0x01, 0x08, 0x2E, 0x2E, 0x00, 0xB6, 0xD0, 0x68,
                                    0x3E, 0x80, 0x2F, 0x0C, 0xA9, 0xFE, 0x64, 0x53, 0x69, 0x7A};

/* ------------------------------------------------------------------ context */
enum kernel_kind { K_NONE, K_OFFICE, K_ODT, K_PDF_R24, K_PDF_R5, K_PDF_R6 };
static const uint32_t DEV_HIT_CAP = 1u << 20;
static const int DEPTH = 3;   /* launches in flight per device before its worker retires the oldest */

/* One device of a context: its stream, its copies of the tables and document constants, its result
 * buffer, and a pinned ring of launch headers the worker thread reads instead of synchronising the stream
 * (a stream sync would drain the launches queued behind the one being polled). */
struct dev_lane {
    int device = 0;
    hipStream_t stream = nullptr;
    dprf_aes_tables *d_tables = nullptr;
    uint32_t *d_enc = nullptr;
    dprf_results *d_res = nullptr;
    uint32_t *d_keys = nullptr;      /* KDF -> check hand-off, 8 words per candidate of one chunk */
    uint32_t *d_slots = nullptr;     /* list mode: [n][DPRF_SLOT_WORDS] */
    uint8_t *d_lens = nullptr;
    size_t slot_cap = 0;
    dprf_results *h_ring = nullptr;  /* DEPTH launch headers + 1 (reset template / final header), pinned */
    hipEvent_t ev[DEPTH][4] = {};    /* per ring slot: start, mid (KDF done), end, header copied */
    dprf_odt_params odt{};           /* .enc -> this device's ciphertext copy */
    double rate = 0;                 /* candidates per ms on this device (last full launch), 0 = unknown */
};

struct dprf_ctx {
    int fmt = 0, flags = 0;
    kernel_kind kind = K_NONE;
    dprf_office_params office{};
    dprf_odt_params odt{};
    dprf_pdf_params pdf{};
    std::vector<uint32_t> odt_words;  /* first min(len,1024) ciphertext bytes, BE words */
    std::vector<dev_lane> lanes;
    uint8_t *h_slots = nullptr;       /* list-mode staging (pinned, portable), shared by the lanes */
    uint8_t *h_lens = nullptr;
    size_t h_cap = 0;
    std::mutex call_mu;               /* one call at a time per context: the lanes' buffers are per call */
};

static const char *kind_name(kernel_kind k) {
    switch (k) {
        case K_OFFICE: return "office_std";
        case K_ODT: return "odf_aes256";
        case K_PDF_R24: return "pdf_r24";
        case K_PDF_R5: return "pdf_r5";
        case K_PDF_R6: return "pdf_r6";
        default: return "none";
    }
}

static int parse_office(dprf_ctx *c, const char *const *f) {
    /* argv mapping brute_force.py:163-173 */
    int salt_len = atoi(f[4]);
    int ev_len = (int)(strlen(f[6]) / 2), evh_len = (int)(strlen(f[7]) / 2);
    int key_bits = atoi(f[3]), hash_size = atoi(f[2]);
    if (salt_len != 16) return fail(DPRF_E_DOMAIN, "office: salt_len %d (office2john asserts 16)", salt_len);
    if (ev_len % 16 || evh_len % 16 || ev_len > 128 || evh_len > 128)
        return fail(DPRF_E_DOMAIN, "office: verifier lengths %d/%d abort the reference's EVP decrypt", ev_len, evh_len);
    if (key_bits < 128) return fail(DPRF_E_DOMAIN, "office: key_bits %d < 128", key_bits);
    std::vector<uint8_t> salt, ev, evh;
    int r;
    if ((r = decode_hex(f[5], salt_len, salt, c->flags, "office salt"))) return r;
    if ((r = decode_hex(f[6], ev_len, ev, c->flags, "office encrypted verifier"))) return r;
    if ((r = decode_hex(f[7], evh_len, evh, c->flags, "office encrypted verifier hash"))) return r;
    if (ev_len != 16 || evh_len != 32) {
        c->flags |= DPRF_FLAG_NEVER_MATCHES;   /* msoffcrypto...c:163,168 */
        return DPRF_OK;
    }
    if (hash_size < 0 || hash_size >= 32)
        return fail(DPRF_E_DOMAIN, "office: verifier_hash_size %d reads past the decrypted hash", hash_size);
    for (int i = 0; i < 4; i++) c->office.salt[i] = be_word(&salt[4 * i]);
    for (int i = 0; i < 4; i++) c->office.ev[i] = be_word(&ev[4 * i]);
    for (int i = 0; i < 8; i++) c->office.evh[i] = be_word(&evh[4 * i]);
    c->office.hash_size = (uint32_t)hash_size;
    c->kind = K_OFFICE;
    return DPRF_OK;
}

static int parse_odt(dprf_ctx *c, const char *const *f) {
    /* argv mapping brute_force.py:175-182 */
    int enc_len = atoi(f[6]);
    if (enc_len < 0 || enc_len % 16)
        return fail(DPRF_E_DOMAIN, "odt: encrypted length %d is not a multiple of 16 (reference aborts)", enc_len);
    std::vector<uint8_t> ck, iv, salt, enc;
    int r;
    if ((r = decode_hex(f[2], 32, ck, c->flags, "odt checksum"))) return r;
    if ((r = decode_hex(f[3], 16, iv, c->flags, "odt iv"))) return r;
    if ((r = decode_hex(f[4], 16, salt, c->flags, "odt salt"))) return r;
    if ((r = decode_hex(f[5], enc_len, enc, c->flags, "odt encrypted file"))) return r;
    for (int i = 0; i < 8; i++) c->odt.checksum[i] = be_word(&ck[4 * i]);
    for (int i = 0; i < 4; i++) c->odt.iv[i] = be_word(&iv[4 * i]);
    for (int i = 0; i < 4; i++) c->odt.salt[i] = be_word(&salt[4 * i]);
    c->odt.enc_len = (uint32_t)enc_len;
    c->odt.hash_len = (uint32_t)std::min(enc_len, 1024);
    const uint32_t nw = std::max<uint32_t>(4u, c->odt.hash_len / 4);
    c->odt_words.assign(nw, 0u);
    for (uint32_t i = 0; i < c->odt.hash_len / 4; i++) c->odt_words[i] = be_word(&enc[4 * i]);
    c->kind = K_ODT;
    return DPRF_OK;
}

static int parse_pdf(dprf_ctx *c, const char *const *f) {
    /* argv mapping brute_force.py:184-197 */
    int V = atoi(f[1]), R = atoi(f[2]), Length = atoi(f[3]), P = atoi(f[4]), meta = atoi(f[5]);
    int id_len = atoi(f[6]), u_len = atoi(f[8]), o_len = atoi(f[10]);
    std::vector<uint8_t> id, u, o;
    int r;
    if ((r = decode_hex(f[7], id_len, id, c->flags, "pdf id"))) return r;
    if ((r = decode_hex(f[9], u_len, u, c->flags, "pdf U"))) return r;
    if ((r = decode_hex(f[11], o_len, o, c->flags, "pdf O"))) return r;
    /* (V,R) whitelist and Length % 8 (pdf...c:89-101) */
    if ((V != 1 && V != 2 && V != 4 && V != 5) || (V == 1 && R != 2) || (V == 2 && R != 3) ||
        (V == 4 && R != 4) || (V == 5 && (R != 5 && R != 6)) || Length % 8 != 0) {
        c->flags |= DPRF_FLAG_NEVER_MATCHES;
        return DPRF_OK;
    }
    dprf_pdf_params &p = c->pdf;
    p.R = (uint32_t)R;
    for (int i = 0; i < 8; i++) p.pad[i] = le_word(PDF_PAD + 4 * i);
    if (R >= 5) {
        if (u_len < 40) return fail(DPRF_E_DOMAIN, "pdf R%d: U shorter than 40 bytes", R);
        for (int i = 0; i < 8; i++) p.u[i] = be_word(&u[4 * i]);
        p.u[8] = le_word(&u[32]);
        p.u[9] = le_word(&u[36]);
        c->kind = R == 5 ? K_PDF_R5 : K_PDF_R6;
        return DPRF_OK;
    }
    int n = Length / 8;
    if (R == 2 && (n < 5 || u_len < 32)) return fail(DPRF_E_DOMAIN, "pdf R2: Length %d / U length %d", Length, u_len);
    if (R >= 3 && ((n != 5 && n != 16) || u_len < 16))
        return fail(DPRF_E_DOMAIN, "pdf R%d: key length %d bytes (EVP_rc4 reads 16 key bytes)", R, n);
    p.n = (uint32_t)n;
    for (int i = 0; i < (R == 2 ? 8 : 4); i++) p.u[i] = le_word(&u[4 * i]);
    /* the document-constant tail of the initial MD5 message (get_initial_md5_hash :352-402) */
    std::vector<uint8_t> msg(PDF_PAD, PDF_PAD + 32);   /* placeholder for the 32 password bytes */
    msg.insert(msg.end(), o.begin(), o.end());
    uint32_t pb = (uint32_t)P;
    for (int i = 0; i < 4; i++) msg.push_back((uint8_t)(pb >> (8 * i)));
    msg.insert(msg.end(), id.begin(), id.end());
    if (R >= 4 && !meta)
        for (int i = 0; i < 4; i++) msg.push_back(0xff);
    uint64_t bits = (uint64_t)msg.size() * 8;
    msg.push_back(0x80);
    while (msg.size() % 64 != 56) msg.push_back(0);
    for (int i = 0; i < 8; i++) msg.push_back((uint8_t)(bits >> (8 * i)));
    size_t tail_words = (msg.size() - 32) / 4;
    if (tail_words > DPRF_PDF_TAIL_WORDS) return fail(DPRF_E_DOMAIN, "pdf: O/ID too long (%zu tail words)", tail_words);
    for (size_t i = 0; i < tail_words; i++) p.tail[i] = le_word(&msg[32 + 4 * i]);
    p.tail_blocks = (uint32_t)(msg.size() / 64 - 1);
    /* MD5(PAD || ID) (get_final_md5_hash :404-434) */
    std::vector<uint8_t> m2(PDF_PAD, PDF_PAD + 32);
    m2.insert(m2.end(), id.begin(), id.end());
    uint8_t h2[16];
    md5_host(m2.data(), m2.size(), h2);
    for (int i = 0; i < 4; i++) p.h2[i] = le_word(h2 + 4 * i);
    c->kind = K_PDF_R24;
    return DPRF_OK;
}

/* Candidates per launch.  A device takes its next chunk from the call's shared cursor sized for about
 * `target_ms` of device time at the rate it measured on its last launch (`init` before the first), a
 * power of two in [lo, hi].  The floors keep whole waves of workgroups on the chip: Office's 2^19 is one
 * full generation of k_office_kdf (256 CUs x 32 waves x 64 lanes); R6's persistent workgroups drain at the
 * end of every launch, so its launches take ~3 s (below). */
struct chunk_policy { uint32_t init, lo, hi; double target_ms; };
#ifndef DPRF_R24_HI_LOG2
#define DPRF_R24_HI_LOG2 30
#endif
/* R6: every launch of the persistent kernel ends in a drain (the last candidates' ~35 remaining rounds with
 * fewer live slots than lanes), so its launches are long: same 2^23-candidate steps measured 2.79 / 2.92 /
 * 3.00 M cand/s with 2^21 / 2^22 / 2^23 per launch (tools/ab_r6_chunk.sh, round 2) */
#ifndef DPRF_R6_LO_LOG2
#define DPRF_R6_LO_LOG2 21
#endif
#ifndef DPRF_R6_HI_LOG2
#define DPRF_R6_HI_LOG2 24
#endif
#ifndef DPRF_R6_TARGET_MS
#define DPRF_R6_TARGET_MS 3000.0
#endif
static chunk_policy policy(kernel_kind k) {
    switch (k) {
        case K_OFFICE: return {1u << 19, 1u << 19, 1u << 20, 400.0};
        case K_ODT: return {1u << 22, 1u << 19, 1u << 23, 300.0};
        case K_PDF_R24: return {1u << 24, 1u << 20, 1u << DPRF_R24_HI_LOG2, 100.0};
        case K_PDF_R5: return {1u << 27, 1u << 22, 1u << 31, 100.0};
        case K_PDF_R6: return {1u << 22, 1u << DPRF_R6_LO_LOG2, 1u << DPRF_R6_HI_LOG2, DPRF_R6_TARGET_MS};
        default: return {1u << 24, 1u << 20, 1u << 24, 100.0};
    }
}
static uint32_t lane_chunk(const dev_lane &L, kernel_kind k) {
    const chunk_policy p = policy(k);
    if (L.rate <= 0) return p.init;
    const double want = L.rate * p.target_ms;
    uint32_t c = p.lo;
    while (c < p.hi && 2.0 * c <= want) c <<= 1;
    return c;
}

/* ------------------------------------------------------------------ ABI: library */
extern "C" int dprf_abi_version(void) { return DPRF_ABI_VERSION; }
extern "C" const char *dprf_last_error(void) { return g_err.c_str(); }

static bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}
extern "C" int dprf_device_list(int *ordinals, int cap) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    int k = 0;
    for (int i = 0; i < n; i++)
        if (is_gfx950(i)) {
            if (ordinals && k < cap) ordinals[k] = i;
            k++;
        }
    return k;
}
extern "C" int dprf_device_count(void) { return dprf_device_list(nullptr, 0); }

/* ------------------------------------------------------------------ ABI: context */
static void lane_free(dev_lane &L) {
    if (hipSetDevice(L.device) != hipSuccess) return;
    if (L.stream) (void)hipStreamSynchronize(L.stream);
    (void)hipFree(L.d_tables);
    (void)hipFree(L.d_enc);
    (void)hipFree(L.d_res);
    (void)hipFree(L.d_slots);
    (void)hipFree(L.d_lens);
    (void)hipFree(L.d_keys);
    if (L.h_ring) (void)hipHostFree(L.h_ring);
    for (auto &s : L.ev)
        for (auto &e : s)
            if (e) (void)hipEventDestroy(e);
    if (L.stream) (void)hipStreamDestroy(L.stream);
    L = dev_lane();
}

extern "C" int dprf_ctx_destroy(dprf_ctx *c) {
    if (!c) return DPRF_OK;
    for (auto &L : c->lanes) lane_free(L);
    if (c->h_slots) (void)hipHostFree(c->h_slots);
    if (c->h_lens) (void)hipHostFree(c->h_lens);
    delete c;
    return DPRF_OK;
}

static int lane_init(dprf_ctx *c, dev_lane &L, int device) {
    L.device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&L.d_tables, sizeof(dprf_aes_tables)));
    HIPCHK(hipMemcpy(L.d_tables, &aes_tables(), sizeof(dprf_aes_tables), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&L.d_res, sizeof(dprf_results) + sizeof(unsigned long long) * DEV_HIT_CAP));
    HIPCHK(hipHostMalloc(&L.h_ring, sizeof(dprf_results) * (DEPTH + 1), hipHostMallocDefault));
    for (auto &s : L.ev)
        for (auto &e : s) HIPCHK(hipEventCreate(&e));
    if (c->kind == K_OFFICE || c->kind == K_ODT)
        HIPCHK(hipMalloc(&L.d_keys, (size_t)8 * sizeof(uint32_t) * policy(c->kind).hi));
    if (c->kind == K_ODT) {
        HIPCHK(hipMalloc(&L.d_enc, c->odt_words.size() * sizeof(uint32_t)));
        HIPCHK(hipMemcpy(L.d_enc, c->odt_words.data(), c->odt_words.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        L.odt = c->odt;
        L.odt.enc = L.d_enc;
    }
    return DPRF_OK;
}

extern "C" int dprf_ctx_create_devices(const char *const *fields, int nfields, const int *devices, int ndev,
                                       dprf_ctx **out) {
    if (!out || !fields || nfields < 1 || !devices || ndev < 1 || ndev > DPRF_MAX_DEVICES)
        return fail(DPRF_E_INVALID, "dprf_ctx_create: null argument or device count %d", ndev);
    *out = nullptr;
    for (int i = 0; i < nfields; i++)
        if (!fields[i]) return fail(DPRF_E_INVALID, "dprf_ctx_create: field %d is NULL", i);
    int nhip = 0;
    if (hipGetDeviceCount(&nhip) != hipSuccess) nhip = 0;
    for (int k = 0; k < ndev; k++)
        if (devices[k] < 0 || devices[k] >= nhip || !is_gfx950(devices[k]))
            return fail(DPRF_E_NODEVICE, "no gfx950 device with ordinal %d (%d HIP devices visible)", devices[k], nhip);
    dprf_ctx *c = new dprf_ctx();
    int r = DPRF_OK;
    const char *tag = fields[0];
    /* parse_verification_data's accepted shapes (brute_force.py:253-260) */
    if (!strcmp(tag, "office") && nfields == 8) { c->fmt = DPRF_FMT_OFFICE; r = parse_office(c, fields); }
    else if (!strcmp(tag, "odt") && nfields == 7) { c->fmt = DPRF_FMT_ODT; r = parse_odt(c, fields); }
    else if (!strcmp(tag, "pdf") && nfields == 12) { c->fmt = DPRF_FMT_PDF; r = parse_pdf(c, fields); }
    else r = fail(DPRF_E_INVALID, "The input data is not supported (tag '%s', %d fields).", tag, nfields);
    c->lanes.resize((size_t)ndev);
    for (int k = 0; r == DPRF_OK && k < ndev; k++) r = lane_init(c, c->lanes[k], devices[k]);
    if (r != DPRF_OK) {
        std::string keep = g_err;
        dprf_ctx_destroy(c);
        g_err = keep;
        return r;
    }
    *out = c;
    return DPRF_OK;
}

extern "C" int dprf_ctx_create(const char *const *fields, int nfields, int device, dprf_ctx **out) {
    if (device == DPRF_ALL_DEVICES) {
        int ords[DPRF_MAX_DEVICES];
        const int n = std::min(dprf_device_list(ords, DPRF_MAX_DEVICES), DPRF_MAX_DEVICES);
        if (n < 1) return fail(DPRF_E_NODEVICE, "no gfx950 device visible");
        return dprf_ctx_create_devices(fields, nfields, ords, n, out);
    }
    return dprf_ctx_create_devices(fields, nfields, &device, 1, out);
}
extern "C" int dprf_ctx_format(const dprf_ctx *c) { return c ? c->fmt : DPRF_E_INVALID; }
extern "C" int dprf_ctx_flags(const dprf_ctx *c) { return c ? c->flags : DPRF_E_INVALID; }
extern "C" const char *dprf_ctx_kernel(const dprf_ctx *c) { return c ? kind_name(c->kind) : "none"; }
extern "C" int dprf_ctx_devices(const dprf_ctx *c, int *ordinals, int cap) {
    if (!c) return fail(DPRF_E_INVALID, "dprf_ctx_devices: null context");
    for (int k = 0; k < (int)c->lanes.size() && k < cap; k++)
        if (ordinals) ordinals[k] = c->lanes[k].device;
    return (int)c->lanes.size();
}

/* ------------------------------------------------------------------ launching */
static hipError_t launch(dprf_ctx *c, dev_lane &L, const dprf_enum &e, uint32_t stop, hipEvent_t mid) {
    const uint32_t cap = DEV_HIT_CAP;
    switch (c->kind) {
        case K_OFFICE: return launch_office(e, c->office, L.d_tables, L.d_res, cap, stop, L.stream, L.d_keys, mid);
        case K_ODT: return launch_odt(e, L.odt, L.d_tables, L.d_res, cap, stop, L.stream, L.d_keys, mid);
        case K_PDF_R24: return launch_pdf_r24(e, c->pdf, L.d_res, cap, stop, L.stream);
        case K_PDF_R5: return launch_pdf_r5(e, c->pdf, L.d_res, cap, stop, L.stream);
        case K_PDF_R6: return launch_pdf_r6(e, c->pdf, L.d_tables, L.d_res, cap, stop, L.stream);
        default: return hipErrorInvalidValue;
    }
}

/* u32 division by d via multiply-high (round-up method): q = (mulhi(n,m) + ((n - mulhi) >> 1)) >> s */
static void fastdiv_magic(uint32_t d, uint32_t &m, uint32_t &s) {
    if (d <= 1) { m = 0; s = 0; return; }
    uint32_t l = 0;
    while ((1ull << l) < d) l++;
    m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
    s = l - 1;
}

/* State of one API call shared by its device workers. */
struct call_state {
    uint64_t total = 0;                  /* candidates of the call                                   */
    uint64_t base = 0;                   /* index of offset 0 (range: start; list: 0)               */
    int stop_on_first = 0;
    std::atomic<uint64_t> next{0};       /* shared chunk cursor (offsets handed out in increasing order) */
    std::atomic<uint64_t> first{~0ull};  /* lowest hit index any device has reported so far          */
    std::atomic<int> err{0};
    std::mutex mu;
    std::string msg;
    void error(int code, const std::string &m) {
        int z = 0;
        if (err.compare_exchange_strong(z, code)) {
            std::lock_guard<std::mutex> g(mu);
            msg = m;
        }
    }
};
static void atomic_min_u64(std::atomic<uint64_t> &a, uint64_t v) {
    uint64_t cur = a.load();
    while (v < cur && !a.compare_exchange_weak(cur, v)) {}
}

struct lane_result {
    std::vector<unsigned long long> hits;
    uint32_t nhits = 0;
    uint64_t first = ~0ull, evaluated = 0, launches = 0, launched = 0;
    double kms = 0, mms = 0;
};

/* The worker of one device: take the next chunk from the shared cursor, launch it, keep DEPTH launches in
 * flight, retire the oldest (timing, its header's lowest hit -> the call's `first`); with stop_on_first stop
 * taking chunks once the next one starts above `first`.  Finally read this device's hits. */
template <class MK>
static void lane_run(dprf_ctx *c, dev_lane &L, call_state &cs, MK &mk, lane_result &out) {
    char buf[600];
    auto hip_fail = [&](const char *what, hipError_t e) {
        char msg[700];   /* `what` may be buf itself */
        snprintf(msg, sizeof msg, "%s (device %d): %s", what, L.device, hipGetErrorString(e));
        cs.error(DPRF_E_HIP, msg);
    };
    hipError_t e = hipSetDevice(L.device);
    if (e != hipSuccess) { hip_fail("hipSetDevice", e); return; }
    dprf_results *fin = L.h_ring + DEPTH;
    memset(fin, 0, sizeof *fin);
    fin->first = ~0ull;
    e = hipMemcpyAsync(L.d_res, fin, sizeof(dprf_results), hipMemcpyHostToDevice, L.stream);
    if (e != hipSuccess) { hip_fail("reset results", e); return; }
    const bool two = c->kind == K_OFFICE || c->kind == K_ODT;
    uint32_t nchunk[DEPTH] = {};
    int head = 0, inq = 0;
    auto retire = [&]() -> hipError_t {
        const int s = head;
        hipError_t r = hipEventSynchronize(L.ev[s][3]);
        if (r != hipSuccess) return r;
        float ms = 0, m = 0;
        (void)hipEventElapsedTime(&ms, L.ev[s][0], L.ev[s][2]);
        if (two) (void)hipEventElapsedTime(&m, L.ev[s][0], L.ev[s][1]);
        else m = ms;
        out.kms += ms;
        out.mms += m;
        out.launches++;
        const unsigned long long f = L.h_ring[s].first;
        if (f != ~0ull) atomic_min_u64(cs.first, f);
        /* the launch's rate (candidates / device ms) sizes this device's next chunks; a launch may have
         * skipped blocks only with stop_on_first after a hit */
        if ((!cs.stop_on_first || f == ~0ull) && ms > 0.05f) L.rate = nchunk[s] / (double)ms;
        head = (head + 1) % DEPTH;
        inq--;
        return hipSuccess;
    };
    const char *failed = nullptr;
    while (cs.err.load() == 0) {
        const uint32_t want = lane_chunk(L, c->kind);
        const uint64_t off = cs.next.fetch_add(want);
        if (off >= cs.total) break;
        if (cs.stop_on_first && cs.base + off > cs.first.load()) break;
        if (inq == DEPTH) {
            if ((e = retire()) != hipSuccess) { failed = "hipEventSynchronize"; break; }
            if (cs.stop_on_first && cs.base + off > cs.first.load()) break;
        }
        const uint32_t n = (uint32_t)std::min<uint64_t>(want, cs.total - off);
        const int s = (head + inq) % DEPTH;
        dprf_enum en;
        memset(&en, 0, sizeof en);
        if ((e = mk(L, en, off, n)) != hipSuccess) { failed = "candidate upload"; break; }
        if ((e = hipEventRecord(L.ev[s][0], L.stream)) != hipSuccess) { failed = "hipEventRecord"; break; }
        if ((e = launch(c, L, en, cs.stop_on_first ? 1u : 0u, two ? L.ev[s][1] : nullptr)) != hipSuccess) {
            snprintf(buf, sizeof buf, "kernel launch (%s)", kind_name(c->kind));
            hip_fail(buf, e);
            break;
        }
        if ((e = hipEventRecord(L.ev[s][2], L.stream)) != hipSuccess ||
            (e = hipMemcpyAsync(&L.h_ring[s], L.d_res, sizeof(dprf_results), hipMemcpyDeviceToHost, L.stream)) != hipSuccess ||
            (e = hipEventRecord(L.ev[s][3], L.stream)) != hipSuccess) { failed = "launch bookkeeping"; break; }
        nchunk[s] = n;
        out.launched += n;
        inq++;
    }
    while (inq > 0) {
        hipError_t r = retire();
        if (r != hipSuccess) { if (!failed) { failed = "hipEventSynchronize"; e = r; } break; }
    }
    if (failed) { hip_fail(failed, e); return; }
    if ((e = hipMemcpyAsync(fin, L.d_res, sizeof(dprf_results), hipMemcpyDeviceToHost, L.stream)) != hipSuccess ||
        (e = hipStreamSynchronize(L.stream)) != hipSuccess) { hip_fail("result header", e); return; }
    if (fin->pad_) {
        snprintf(buf, sizeof buf, "%s kernel flagged an internal error (0x%x) on device %d", kind_name(c->kind),
                 fin->pad_, L.device);
        cs.error(DPRF_E_HIP, buf);
        return;
    }
    out.nhits = fin->nhits;
    out.first = fin->first;
    out.evaluated = out.launched - fin->skipped;
    const uint32_t ncopy = std::min<uint32_t>(out.nhits, DEV_HIT_CAP);
    out.hits.resize(ncopy);
    if (ncopy &&
        (e = hipMemcpy(out.hits.data(), (char *)L.d_res + offsetof(dprf_results, hits),
                       ncopy * sizeof(unsigned long long), hipMemcpyDeviceToHost)) != hipSuccess) {
        hip_fail("hit list", e);
        return;
    }
    std::sort(out.hits.begin(), out.hits.end());
    if (out.nhits > DEV_HIT_CAP && out.first != ~0ull && out.hits[0] != out.first) {
        /* the device buffer overflowed: keep the lowest hit */
        out.hits.insert(out.hits.begin(), out.first);
        out.hits.pop_back();
    }
}

/* Run a call over every device of the context: one worker thread per device (the calling thread serves the
 * first), then merge the devices' hits. */
template <class MK>
static int run_call(dprf_ctx *c, call_state &cs, MK mk, uint64_t *hits, int64_t cap, int64_t *nhits,
                    dprf_stats *stats, std::chrono::steady_clock::time_point t0) {
    const size_t nd = c->lanes.size();
    std::vector<lane_result> res(nd);
    std::vector<std::thread> th;
    for (size_t k = 1; k < nd; k++) th.emplace_back([&, k] { lane_run(c, c->lanes[k], cs, mk, res[k]); });
    lane_run(c, c->lanes[0], cs, mk, res[0]);
    for (auto &t : th) t.join();
    if (cs.err.load() != 0) return fail(cs.err.load(), "%s", cs.msg.c_str());
    std::vector<unsigned long long> all;
    uint64_t nh = 0, evaluated = 0, launches = 0;
    double kms = 0, mms = 0;
    for (auto &r : res) {
        all.insert(all.end(), r.hits.begin(), r.hits.end());
        nh += r.nhits;
        evaluated += r.evaluated;
        launches += r.launches;
        kms += r.kms;
        mms += r.mms;
    }
    std::sort(all.begin(), all.end());
    if (hits)
        for (int64_t i = 0; i < cap && i < (int64_t)all.size(); i++) hits[i] = all[i];
    if (nhits) *nhits = (int64_t)nh;
    if (stats) {
        stats->candidates = evaluated;
        stats->launches = launches;
        stats->kernel_ms = kms;
        stats->main_kernel_ms = mms;
        stats->wall_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        stats->stopped_early = evaluated < cs.total ? 1u : 0u;
        stats->devices = (uint32_t)nd;
    }
    return DPRF_OK;
}

static void empty_result(uint64_t count, int64_t *nhits, dprf_stats *stats, size_t nd) {
    if (nhits) *nhits = 0;
    if (stats) {
        memset(stats, 0, sizeof *stats);
        stats->candidates = count;
        stats->devices = (uint32_t)nd;
    }
}

/* ------------------------------------------------------------------ ABI: range mode */
extern "C" int dprf_search_range(dprf_ctx *c, const uint8_t *charset, int cslen, int pwlen, uint64_t start,
                                 uint64_t count, int stop_on_first, uint64_t *hits, int64_t cap, int64_t *nhits,
                                 dprf_stats *stats) {
    if (!c || !charset) return fail(DPRF_E_INVALID, "dprf_search_range: null argument");
    if (cslen < 1 || cslen > 256) return fail(DPRF_E_CHARSET, "charset length %d", cslen);
    if (pwlen < 1 || pwlen > DPRF_MAX_PW_RANGE) return fail(DPRF_E_PWLEN, "range password length %d (1..%d)", pwlen, DPRF_MAX_PW_RANGE);
    for (int i = 0; i < cslen; i++) {
        if (charset[i] == 0) return fail(DPRF_E_CHARSET, "charset contains NUL (the reference passes candidates via argv)");
        if (c->fmt == DPRF_FMT_OFFICE && charset[i] >= 0x80)
            return fail(DPRF_E_CHARSET, "Office range mode needs an ASCII charset (UTF-16LE of single bytes)");
    }
    /* keyspace bound: start + count <= cslen^pwlen */
    long double space = 1;
    for (int i = 0; i < pwlen; i++) space *= cslen;
    if ((long double)start + (long double)count > space)
        return fail(DPRF_E_INVALID, "range [%llu, +%llu) exceeds the keyspace %d^%d", (unsigned long long)start,
                    (unsigned long long)count, cslen, pwlen);
    std::lock_guard<std::mutex> call_lock(c->call_mu);
    const auto t0 = std::chrono::steady_clock::now();
    if (c->kind == K_NONE || count == 0) { empty_result(count, nhits, stats, c->lanes.size()); return DPRF_OK; }
    uint32_t m, s;
    fastdiv_magic((uint32_t)cslen, m, s);
    call_state cs;
    cs.total = count;
    cs.base = start;
    cs.stop_on_first = stop_on_first;
    return run_call(
        c, cs,
        [&](dev_lane &, dprf_enum &e, uint64_t off, uint32_t n) -> hipError_t {
            e.start = start + off;
            e.count = n;
            e.mode = 0;
            e.pwlen = (uint32_t)pwlen;
            e.cslen = (uint32_t)cslen;
            e.div_m = m;
            e.div_s = s;
            uint64_t v = e.start;
            for (int p = pwlen - 1; p >= 0; p--) { e.sdig[p] = (uint8_t)(v % (uint64_t)cslen); v /= (uint64_t)cslen; }
            memcpy(e.charset, charset, (size_t)cslen);
            return hipSuccess;
        },
        hits, cap, nhits, stats, t0);
}

/* ------------------------------------------------------------------ ABI: list mode */
/* UTF-8 -> UTF-16LE as iconv("UTF16LE","UTF8") (msoffcrypto...c:275-336); -1 on invalid input */
static int utf8_to_utf16le(const uint8_t *s, size_t n, uint8_t *out, size_t cap) {
    size_t o = 0;
    for (size_t i = 0; i < n;) {
        uint32_t cp;
        int k;
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
        if ((k == 2 && cp < 0x80) || (k == 3 && cp < 0x800) || (k == 4 && (cp < 0x10000 || cp > 0x10FFFF))) return -1;
        if (cp >= 0xD800 && cp <= 0xDFFF) return -1;
        if (cp >= 0x10000) {
            if (o + 4 > cap) return -2;
            uint32_t v = cp - 0x10000, hi = 0xD800 | (v >> 10), lo = 0xDC00 | (v & 0x3FF);
            out[o++] = (uint8_t)hi; out[o++] = (uint8_t)(hi >> 8); out[o++] = (uint8_t)lo; out[o++] = (uint8_t)(lo >> 8);
        } else {
            if (o + 2 > cap) return -2;
            out[o++] = (uint8_t)cp; out[o++] = (uint8_t)(cp >> 8);
        }
        i += k;
    }
    return (int)o;
}

/* One candidate into its 64-byte slot, with the per-format conversion the reference's verifier applies
 * before hashing: UTF-16LE (Office, iconv at msoffcrypto...c:80), 32-byte truncation (PDF R<=4,
 * pdf...c:137), 127-byte truncation (PDF R5, :197-200).  Returns the slot's byte length or DPRF_E_*. */
static int pack_candidate(const dprf_ctx *c, const uint8_t *pw, size_t len, uint8_t *dst) {
    const size_t SB = DPRF_SLOT_WORDS * 4;
    memset(dst, 0, SB);
    if (memchr(pw, 0, len)) return DPRF_E_INVALID;              /* argv cannot carry a NUL */
    if (c->fmt == DPRF_FMT_OFFICE) {
        if (len == 0) return DPRF_E_DOMAIN;                     /* reference UB on the iconv path */
        const int u = utf8_to_utf16le(pw, len, dst, SB);
        if (u == -1) return DPRF_E_DOMAIN;                      /* iconv fails on invalid UTF-8 */
        if (u < 0) return DPRF_E_PWLEN;
        return u;
    }
    if (c->kind == K_PDF_R24 && len > 32) len = 32;
    if (c->kind == K_PDF_R5 && len > 127) len = 127;
    if (len > SB) return DPRF_E_PWLEN;
    memcpy(dst, pw, len);
    return (int)len;
}
static const char *status_text(int code) {
    switch (code) {
        case DPRF_E_INVALID: return "contains NUL (argv cannot carry it)";
        case DPRF_E_DOMAIN: return "empty or invalid UTF-8 Office password (the reference's iconv path fails)";
        case DPRF_E_PWLEN: return "longer than the kernels' 64-byte slot (32 UTF-16 code units for Office)";
        default: return "invalid";
    }
}

extern "C" int dprf_list_status(const dprf_ctx *c, const uint8_t *blob, const uint64_t *offsets, int64_t n,
                                int8_t *status) {
    if (!c || n < 0 || (n > 0 && (!blob || !offsets))) return fail(DPRF_E_INVALID, "dprf_list_status: bad argument");
    uint8_t slot[DPRF_SLOT_WORDS * 4];
    int64_t bad = 0;
    for (int64_t k = 0; k < n; k++) {
        int r = offsets[k + 1] < offsets[k] ? DPRF_E_INVALID
                                            : pack_candidate(c, blob + offsets[k], (size_t)(offsets[k + 1] - offsets[k]), slot);
        r = r < 0 ? r : 0;
        if (status) status[k] = (int8_t)r;
        bad += r < 0;
    }
    return (int)std::min<int64_t>(bad, INT32_MAX);
}

extern "C" int dprf_verify_list(dprf_ctx *c, const uint8_t *blob, const uint64_t *offsets, int64_t n,
                                int stop_on_first, uint64_t *hits, int64_t cap, int64_t *nhits, dprf_stats *stats) {
    if (!c || (n > 0 && (!blob || !offsets)) || n < 0) return fail(DPRF_E_INVALID, "dprf_verify_list: bad argument");
    std::lock_guard<std::mutex> call_lock(c->call_mu);
    const auto t0 = std::chrono::steady_clock::now();
    const size_t SB = DPRF_SLOT_WORDS * 4;
    if ((size_t)n > c->h_cap) {
        const size_t want = std::max<size_t>((size_t)n, 2 * c->h_cap);
        if (c->h_slots) (void)hipHostFree(c->h_slots);
        if (c->h_lens) (void)hipHostFree(c->h_lens);
        c->h_slots = nullptr;
        c->h_lens = nullptr;
        c->h_cap = 0;
        HIPCHK(hipHostMalloc(&c->h_slots, want * SB, hipHostMallocPortable));
        HIPCHK(hipHostMalloc(&c->h_lens, want, hipHostMallocPortable));
        c->h_cap = want;
    }
    for (int64_t k = 0; k < n; k++) {
        if (offsets[k + 1] < offsets[k]) return fail(DPRF_E_INVALID, "offsets not monotone at %lld", (long long)k);
        const int r = pack_candidate(c, blob + offsets[k], (size_t)(offsets[k + 1] - offsets[k]), c->h_slots + (size_t)k * SB);
        if (r < 0) return fail(r, "candidate %lld: %s", (long long)k, status_text(r));
        c->h_lens[k] = (uint8_t)r;
    }
    if (c->kind == K_NONE || n == 0) { empty_result((uint64_t)n, nhits, stats, c->lanes.size()); return DPRF_OK; }
    call_state cs;
    cs.total = (uint64_t)n;
    cs.base = 0;
    cs.stop_on_first = stop_on_first;
    return run_call(
        c, cs,
        [&](dev_lane &L, dprf_enum &e, uint64_t off, uint32_t cnt) -> hipError_t {
            hipError_t r;
            if (L.slot_cap < (size_t)n) {   /* first chunk of the call on this device: nothing in flight */
                (void)hipFree(L.d_slots);
                (void)hipFree(L.d_lens);
                L.d_slots = nullptr;
                L.d_lens = nullptr;
                L.slot_cap = 0;
                if ((r = hipMalloc(&L.d_slots, (size_t)n * SB)) != hipSuccess) return r;
                if ((r = hipMalloc(&L.d_lens, (size_t)n)) != hipSuccess) return r;
                L.slot_cap = (size_t)n;
            }
            /* this chunk's slots only: a device uploads what it verifies */
            if ((r = hipMemcpyAsync((uint8_t *)L.d_slots + off * SB, c->h_slots + off * SB, (size_t)cnt * SB,
                                    hipMemcpyHostToDevice, L.stream)) != hipSuccess)
                return r;
            if ((r = hipMemcpyAsync(L.d_lens + off, c->h_lens + off, cnt, hipMemcpyHostToDevice, L.stream)) != hipSuccess)
                return r;
            e.start = off;
            e.count = cnt;
            e.mode = 1;
            e.pwlen = *std::max_element(c->h_lens + off, c->h_lens + off + cnt);
            e.slots = L.d_slots;
            e.lens = L.d_lens;
            return hipSuccess;
        },
        hits, cap, nhits, stats, t0);
}

/* oracle.h -- CPU restatement of the reference verifiers (TEST INFRASTRUCTURE ONLY).
 *
 * This header and oracle.c restate, in plain C with their own FIPS/RFC primitives, what the
 * reference's three verifier executables compute:
 *   - /root/reference/src/ms-offcrypto-impl/msoffcrypto_password_verifier.c  verify() :56-191
 *   - /root/reference/src/odt-impl/odt_password_verifier.c                     verify() :51-126
 *   - /root/reference/src/pdf-impl/pdf_password_verifier.c                     verify() :64-192,
 *       verify_user_r5() :194-221, pdf_compute_hardened_hash_r6() :226-291
 * and the engine's argv mapping (brute_force.py:163-197) and field split (brute_force.py:245-264).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.  The
 * product (dprf_amd/, libdprf.so) never links or calls it: it is the checker, not the thing measured.
 * Parity of this restatement is pinned against the reference itself, built from its own sources
 * into oracle/_ref by oracle/ref.mk (tests/golden/make_golden.py), and against standard KATs.
 */
#ifndef DPRF_ORACLE_H
#define DPRF_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- primitives (KAT-tested) ---- */
void orc_sha1(const uint8_t *m, size_t n, uint8_t out[20]);
void orc_sha256(const uint8_t *m, size_t n, uint8_t out[32]);
void orc_sha384(const uint8_t *m, size_t n, uint8_t out[48]);
void orc_sha512(const uint8_t *m, size_t n, uint8_t out[64]);
void orc_md5(const uint8_t *m, size_t n, uint8_t out[16]);
void orc_aes_encrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]);
void orc_aes_decrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]);
void orc_rc4(const uint8_t *key, int keylen, const uint8_t *in, size_t n, uint8_t *out);
void orc_pbkdf2_hmac_sha1(const uint8_t *pw, size_t pwlen, const uint8_t *salt, size_t saltlen,
                          uint32_t iters, uint8_t *out, size_t outlen);

/* BN_hex2bn + BN_bn2bin (str_to_uchar, msoffcrypto...c:340-349): returns the number of bytes the
 * reference writes (leading 0x00 bytes dropped), writes them left-aligned into out[0..cap). */
int orc_bn_hex_decode(const char *hex, uint8_t *out, int cap);

/* ---- per-document context built from parse_verification_data's field array ---- */
typedef struct orc_ctx orc_ctx;

#define ORC_FMT_OFFICE 1
#define ORC_FMT_ODT 2
#define ORC_FMT_PDF 3

/* ctx flags */
#define ORC_FLAG_NEVER_MATCHES 1      /* reference verify() returns 0 for every candidate (gates) */
#define ORC_FLAG_REF_NONDETERMINISTIC 2 /* a hex field decodes short in the reference (leading 00) */

int orc_ctx_create(const char *const *fields, int nfields, orc_ctx **out);
void orc_ctx_destroy(orc_ctx *ctx);
int orc_ctx_format(const orc_ctx *ctx);
int orc_ctx_flags(const orc_ctx *ctx);

/* 1 = the reference verifier exits 1 ("found"), 0 = exits 0, <0 = outside the parity domain. */
int orc_verify(const orc_ctx *ctx, const uint8_t *pw, int len);

/* Full hit set over [start, start+count) of charset^pwlen in itertools.product order
 * (brute_force.py:205): returns #hits (may exceed cap; first cap indices written in ascending order). */
int64_t orc_search_range(const orc_ctx *ctx, const uint8_t *charset, int cslen, int pwlen,
                         uint64_t start, uint64_t count, int nthreads, uint64_t *hits, int64_t cap);

/* Verdict per candidate of an explicit list (client payload path, brute_force.py:82-104). */
int orc_verify_list(const orc_ctx *ctx, const uint8_t *blob, const uint64_t *offsets, int64_t n,
                    int nthreads, int8_t *verdicts);

/* Intermediates printed by the reference's -v mode (for golden comparison).  Returns bytes written. */
int orc_intermediates(const orc_ctx *ctx, const uint8_t *pw, int len, uint8_t *out, int cap);

/* Primitive work counters for one verify() (roofline accounting):
 * [0] SHA1c [1] SHA256c [2] SHA512c [3] MD5c [4] AES-128 enc blocks [5] AES-256 dec blocks
 * [6] RC4 KSA [7] RC4 PRGA bytes [8] AES-128 key expansions [9] AES-256 key expansions */
#define ORC_NCOUNT 10
int orc_work_counts(const orc_ctx *ctx, const uint8_t *pw, int len, uint64_t counts[ORC_NCOUNT]);

#ifdef __cplusplus
}
#endif
#endif

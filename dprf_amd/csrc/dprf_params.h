/* dprf_params.h -- kernel-argument structs shared by the host (dprf_host.cpp) and the gfx950 kernels
 * (dprf_kernels.hip).  Plain C layout; everything a kernel needs about one document is folded here
 * once per context, never per candidate.  Word conventions: "BE" = the 32-bit big-endian words that
 * SHA-1/SHA-2/AES operate on; "LE" = little-endian words (MD5, RC4 byte order, candidate bytes). */
#ifndef DPRF_PARAMS_H
#define DPRF_PARAMS_H
#include <stdint.h>

#define DPRF_SLOT_WORDS 16          /* list-mode candidate slot: 64 bytes, LE-packed */
#define DPRF_MAX_RANGE_LEN 32
#define DPRF_R6_MAX_LONG 176        /* PDF R6 candidates: data[(128 + 64 + 48) * 64] holds 64 x (pw || K[0:64]) only up
                                       to 176 bytes (pdf...c:228); longer ones abort the reference (stack smashing) */

/* Candidate source for one launch.  Range mode: candidate g of the launch is global keyspace index
 * start + g, spelled over charset in itertools.product order.  List mode: candidate g is slot
 * start + g of the device candidate buffer.  Long-list mode (round 4): candidate g is record start + g of a packed
 * blob of candidates longer than a slot -- k_long_prehash hashes the record's first message (Office H0, the ODF
 * start key, PDF R5's whole hash, R6's K0) into `keys`, and the format's kernels continue from there. */
struct dprf_enum {
    uint64_t start;
    uint32_t count;
    uint32_t mode;                  /* 0 range, 1 list, 2 long list */
    uint32_t pwlen;                 /* range: fixed length (bytes); list / long list: longest candidate of the launch */
    uint32_t cslen;
    uint32_t div_m;                 /* u32 division by cslen: q = (mulhi(n,m) + ((n-mulhi)>>1)) >> s */
    uint32_t div_s;
    uint8_t sdig[DPRF_MAX_RANGE_LEN];   /* base-cslen digits of start, most significant first */
    uint8_t charset[256];
    const uint32_t *slots;          /* list: [n][DPRF_SLOT_WORDS] LE words; long list: the record blob (LE words) */
    const uint8_t *lens;            /* list: [n] byte lengths */
    const uint64_t *loff;           /* long list: [n] word offset of each record in the blob (16-byte aligned)    */
    const uint32_t *llen;           /* long list: [n] byte length of each record                                  */
    uint32_t *keys;                 /* long list: [8][count] prehash output (chunk-local), read by the next kernel */
    /* multi-device stop_on_first calls only (round 6, dprf_hits.h), else null: host-mapped words */
    unsigned long long *hit_mirror;         /* this device lane's lowest hit, lowered by its kernels             */
    const unsigned long long *xfirst;       /* the lowest hit any device of the call has reported (host-kept)    */
};

/* Long-list prehash (k_long_prehash): the first message of the format's verify() over a record of any length. */
#define DPRF_LONG_SHA1_SALT16 1     /* Office H0 = SHA1(salt[0:16] || UTF16LE(pw)) (msoffcrypto...c:94-101) -> keys[5] */
#define DPRF_LONG_SHA256 2          /* ODF start key = SHA256(pw) (odt...c:78-79)                       -> keys[8] */
#define DPRF_LONG_SHA256_SALT8 3    /* R6 K0 = SHA256(pw || salt8) (pdf...c:240-245)                    -> keys[8] */
#define DPRF_LONG_R5 4              /* R5: SHA256(pw[:127] || salt8) == U[0:32] (pdf...c:194-221)       -> hits    */
struct dprf_long_params {
    uint32_t alg;                   /* DPRF_LONG_*                                                          */
    uint32_t prefix[4];             /* SHA1_SALT16: the salt as BE words (message words 0..3)               */
    uint32_t suffix[2];             /* SALT8 / R5: the 8 salt bytes as LE words, appended after the record  */
    uint32_t target[8];             /* R5: U[0:32] as BE words                                              */
};

/* Device results of one API call (accumulated over its launches). */
struct dprf_results {
    uint32_t nhits;                 /* total hits (may exceed cap) */
    uint32_t stop;                  /* set by a hit when stop_on_first */
    uint32_t cursor;                /* work cursor of persistent kernels (PDF R6), reset per launch */
    uint32_t pad_;                  /* error flags set by a kernel, 0 = none: 1 PDF R6 scheduler watchdog, 2 / 4 / 8 an
                                       asm block's LDS-address assumption broken (R2-R4 S-box area, ODF check table,
                                       R6 tables) */
    unsigned long long first;       /* lowest hit index (atomicMin), ~0 if none */
    unsigned long long skipped;     /* candidates of launched chunks NOT evaluated: stop_on_first blocks
                                       skipped above the lowest hit (rare: one atomic per skipped block, none
                                       per evaluated block -- a per-block counter on this line made every
                                       block's `first` load wait behind the atomics, -25 % on PDF R2) */
    unsigned long long hits[1];     /* [cap] */
};

/* AES tables, generated on the host from the GF(2^8) definition (FIPS 197 5.1.1) and copied to LDS by
 * each kernel that needs them. */
struct dprf_aes_tables {
    uint32_t te0[256];              /* forward T-table, BE column (S[x]*{02,01,01,03}) */
    uint32_t td0[256];              /* inverse T-table, BE column (Si[x]*{0e,09,0d,0b}) */
    uint8_t sbox[256];
    uint8_t inv_sbox[256];
};

/* Office: msoffcrypto_password_verifier.c:56-191 */
struct dprf_office_params {
    uint32_t salt[4];               /* BE words of salt[0:16] (:95) */
    uint32_t ev[4];                 /* encrypted verifier, BE */
    uint32_t evh[8];                /* encrypted verifier hash (32 B), BE */
    uint32_t hash_size;             /* byte of dec(evh) that must be 0 (:168) */
};

/* ODT: odt_password_verifier.c:51-126 */
struct dprf_odt_params {
    uint32_t checksum[8];           /* BE */
    uint32_t iv[4];                 /* BE */
    uint32_t salt[4];               /* BE */
    uint32_t enc_len;               /* bytes; multiple of 16 */
    uint32_t hash_len;              /* min(enc_len, 1024) */
    const uint32_t *enc;            /* device: first hash_len bytes of ciphertext, BE words */
};

/* PDF: pdf_password_verifier.c:64-291 */
#define DPRF_PDF_TAIL_WORDS 64
struct dprf_pdf_params {
    uint32_t R;                     /* 2..6 */
    uint32_t n;                     /* Length / 8 (R<=4) */
    uint32_t u[12];                 /* R<=4: U[0:32] LE words; R5/R6: U[0:32] BE words + salt BE */
    uint32_t h2[4];                 /* R3/R4: MD5(PAD || ID), LE (pdf...c:167) */
    uint32_t pad[8];                /* the 32-byte password padding, LE */
    uint32_t tail_blocks;           /* MD5 blocks after the first (initial hash, :352-402) */
    uint32_t tail[DPRF_PDF_TAIL_WORDS]; /* LE words of O||LE32(P)||ID[||FFFFFFFF] + MD5 padding,
                                           starting at message byte 32 */
};

#endif

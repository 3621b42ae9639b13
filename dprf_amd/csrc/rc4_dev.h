/* rc4_dev.h -- RC4 on gfx950 with one 256-byte S-box per lane in LDS (PDF R2-R4, pdf_password_verifier.c:157-176;
 * shared by dprf_kernels.hip and the tools/ micro-benchmarks).  Requires dev_crypto.h. */
#ifndef DPRF_RC4_DEV_H
#define DPRF_RC4_DEV_H
#include "dev_crypto.h"
#include "rc4_ksa_asm.h"

/* RC4 state: one 256-byte S-box per lane in LDS, laid out so that lane l owns bank l%32 for every
 * byte: S[i] of lane l lives at wave_base + (i>>2)*256 + l*4 + (i&3).  Byte reads/writes of a wave
 * therefore never conflict, whatever i/j each lane holds.  16 KiB per wave: 9 such waves fit the ~152 KiB a
 * CU allocates (tools/lds_occ.hip). */
#define RC4_WAVE_BYTES 16384
/* Address of S[j & 0xff] = ((j & 0xfc) << 6) | (j & 3) | lanebase in two half-rate instructions: (j & 3) | lanebase, then byte 1 <- (j & 0xff) >> 2 by an SDWA shift
 * that keeps the other bytes (lanebase < 256); any j (only its low byte counts).  tools/rc4_bench.hip
 * variant 9: +3.6% on the R3/R4 KSA.  Used by every KSA and PRGA step. */
DEVI uint32_t rc4_addr_sdwa(uint32_t j, uint32_t lanebase) {
    uint32_t t = (j & 3u) | lanebase;
    asm("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
        : "+v"(t) : "v"(j));
    return t;
}
DEVI uint32_t lds_ld8(const uint8_t *base, uint32_t a) { return base[a]; }
DEVI void lds_st8(uint8_t *base, uint32_t a, uint32_t v) { base[a] = (uint8_t)v; }

/* S = identity for every lane of the wave: dword w of lane l is at S + 256 w + 4 l, exactly the address
 * ds_write_addtid_b32 forms from M0 + offset + 4 * lane, so the 64 stores carry no address VGPR.  One asm
 * block: the values come from an add chain the compiler cannot hoist out of the pass loop as 64 literal
 * VGPRs; M0 is reserved to the compiler, so the block restores it. */
DEVI void rc4_identity(uint8_t *S) {
    /* wave-uniform (the box of a wave); readfirstlane so a per-wave offset computed in VGPRs can feed M0 */
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(__attribute__((address_space(3))) uint8_t *)S);
    uint32_t t, m0save;
#define RC4_ID_W(o) "ds_write_addtid_b32 %0 offset:" #o "\n\tv_add_u32 %0, 0x4040404, %0\n\t"
    asm volatile(
        "s_mov_b32 %1, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "v_mov_b32 %0, 0x3020100\n\t"
        RC4_ID_W(0) RC4_ID_W(256) RC4_ID_W(512) RC4_ID_W(768) RC4_ID_W(1024) RC4_ID_W(1280) RC4_ID_W(1536) RC4_ID_W(1792)
        RC4_ID_W(2048) RC4_ID_W(2304) RC4_ID_W(2560) RC4_ID_W(2816) RC4_ID_W(3072) RC4_ID_W(3328) RC4_ID_W(3584) RC4_ID_W(3840)
        RC4_ID_W(4096) RC4_ID_W(4352) RC4_ID_W(4608) RC4_ID_W(4864) RC4_ID_W(5120) RC4_ID_W(5376) RC4_ID_W(5632) RC4_ID_W(5888)
        RC4_ID_W(6144) RC4_ID_W(6400) RC4_ID_W(6656) RC4_ID_W(6912) RC4_ID_W(7168) RC4_ID_W(7424) RC4_ID_W(7680) RC4_ID_W(7936)
        RC4_ID_W(8192) RC4_ID_W(8448) RC4_ID_W(8704) RC4_ID_W(8960) RC4_ID_W(9216) RC4_ID_W(9472) RC4_ID_W(9728) RC4_ID_W(9984)
        RC4_ID_W(10240) RC4_ID_W(10496) RC4_ID_W(10752) RC4_ID_W(11008) RC4_ID_W(11264) RC4_ID_W(11520) RC4_ID_W(11776) RC4_ID_W(12032)
        RC4_ID_W(12288) RC4_ID_W(12544) RC4_ID_W(12800) RC4_ID_W(13056) RC4_ID_W(13312) RC4_ID_W(13568) RC4_ID_W(13824) RC4_ID_W(14080)
        RC4_ID_W(14336) RC4_ID_W(14592) RC4_ID_W(14848) RC4_ID_W(15104) RC4_ID_W(15360) RC4_ID_W(15616) RC4_ID_W(15872) RC4_ID_W(16128)
        "s_mov_b32 m0, %1"
        : "=&v"(t), "=&s"(m0save)
        : "s"(base)
        : "memory");
#undef RC4_ID_W
}

/* KSA with an NK-byte key held LE-packed in k[4].
 *
 * Step i: j += S[i] + K[i % NK]; swap(S[i], S[j]).  Positions i0 = 2q, i1 = 2q + 1 (one u16 of this lane's
 * S-box) form group q, read with one LDS load W that was issued at the end of group q-1:
 *  - step 0: v0 = S[i0] = byte 0 of W; j += v0 + key byte; x0 = S[j] is read and S[j] = v0 stored at once;
 *  - step 1: v1 = byte 1 of W, or v0 if step 0 swapped into i1; x1 = S[j] read, S[j] = v1 stored;
 *  - the S[i] sides are NOT stored yet: the next group's W is read first (after both S[j] stores, the only
 *    stores that can touch its positions), and only then S[i0] = (v1 if step 1 hit i0, else x0) and
 *    S[i1] = x1 (x0 instead when step 1 read i0, whose store was still pending) -- one u16 store, LLVM merges
 *    the two.  The next group's first S[j] read comes after that store, so it needs no repair.
 * The wave waits on LDS once per group: for x1, with W right behind it.
 *
 * History (tools/rc4_bench.hip, tools/ab_libs.sh): until late round 2 each S[i] store was
 * deferred by one step only (stored at the next step, the read repaired when it hit i) and W was read after
 * the group's stores, so a group waited twice -- for W, then for x0 at the next step's deferred store, a
 * few instructions after its read: R3/R4 513 M, R2 10.2 G cand/s.  Group-deferred with the W read pinned
 * ahead of the stores: 561 M / 11.3 G.  Without the pin LLVM sinks the W read below the stores (it can
 * prove they do not alias), and the second wait is back: 494 M.  The same with dword groups (G = 4: 12
 * compare-selects per 4 steps) 424 M / 8.6 G: VALU-bound. */
template <int NK>
DEVI void rc4_ksa(uint8_t *S, uint32_t lanebase, const uint32_t k[4]) {
    rc4_identity(S);
    uint32_t kb[NK];
#pragma unroll
    for (int q = 0; q < NK; q++) kb[q] = (k[q >> 2] >> (8 * (q & 3))) & 0xffu;
    uint32_t j = 0;                             /* only its low byte is meaningful */
    uint32_t W = 0x0100u;                       /* group 0 is the identity */
#pragma unroll
    for (int q = 0; q < 128; q++) {
        const uint32_t i0 = 2u * q, i1 = i0 + 1u;
        const uint32_t p0 = ((i0 >> 2) << 8) + (i0 & 3u) + lanebase;
        const uint32_t v0 = W & 0xffu;
        j = j + v0 + kb[i0 % NK];
        const uint32_t a0 = rc4_addr_sdwa(j, lanebase);
        /* m0, m1 are used only in compares, which LLVM folds into SDWA byte selects of j */
        const uint32_t m0 = j & 0xffu;
        const uint32_t x0 = lds_ld8(S, a0);
        lds_st8(S, a0, v0);
        const uint32_t v1 = (m0 == i1) ? v0 : (W >> 8);
        j = j + v1 + kb[i1 % NK];
        const uint32_t a1 = rc4_addr_sdwa(j, lanebase);
        const uint32_t m1 = j & 0xffu;
        uint32_t x1 = lds_ld8(S, a1);
        lds_st8(S, a1, v1);
        if (q < 127) {
            const uint32_t n = i0 + 2u;
            W = *(const uint16_t *)(S + ((n >> 2) << 8) + (n & 3u) + lanebase);
            /* keep the read ahead of the deferred stores (they wait for x1; W must already be in flight) */
            __builtin_amdgcn_sched_barrier(0);
        }
        const bool hit = m1 == i0;
        x1 = hit ? x0 : x1;
        lds_st8(S, p0, hit ? v1 : x0);
        lds_st8(S, p0 + 1u, x1);
    }
}

/* The same KSA as one generated inline-asm block (rc4_ksa_asm.h, tools/gen_rc4_ksa_asm.py: the schedule above in
 * 11 VALU instructions per group of two steps instead of the 16-17 LLVM emits, byte selects as SDWA operands).
 * sbase: LDS address of the wave's 16 KiB area, low 16 bits zero (the SDWA byte-1 insert of the S[j] address
 * overwrites bits 8-15 of lanebase; the caller checks); lanebase = sbase + 4 * lane.  Writes the identity itself
 * and returns with no LDS operation in flight.  kb: the key registers rc4_kb_init makes. */

/* Key registers of the asm KSA from the LE-packed key k[4]: register q holds key byte q in byte 0 (anything above
 * it: the block reads byte 0 only).  Only byte 0 changes when a caller XORs a pass constant < 256 into every
 * register (R3/R4's key ^ x). */
template <int NK>
DEVI void rc4_kb_init(const uint32_t k[4], uint32_t kb[NK]) {
#pragma unroll
    for (int q = 0; q < NK; q++) kb[q] = k[q >> 2] >> (8 * (q & 3));
}

template <int NK>
DEVI void rc4_ksa_asm_kb(uint32_t sbase, uint32_t lanebase, const uint32_t kb[NK]) {
    static_assert(NK == 5 || NK == 16, "rc4_ksa_asm.h holds the 5- and 16-byte key schedules");
    uint32_t j, W, x0, x1, v1, a0, a1, m, st, m0s, wn;
    /* operands the shipped schedule does not read (%8, %11-%15, %18-%20): kept so that the block's register
     * assignment -- and with it the kernel's machine code -- is the one measured (rounds 3-5 variants used them) */
    uint64_t c0, c1, c2, c3, h0;
    const uint32_t l4 = lanebase - sbase;                /* 4 * lane */
    const uint32_t ia = sbase + ((l4 >> 6) << 8) + ((l4 & 60u) << 2);
    const uint32_t d0 = 0x03020100u + 0x04040404u * (l4 >> 6);
    const uint64_t c16 = 0x1010101010101010ull;
#define RC4_KSA_OUTS                                                                                               \
    "=&v"(j), "=&v"(W), "=&v"(x0), "=&v"(x1), "=&v"(v1), "=&v"(a0), "=&v"(a1), "=&v"(m), "=&s"(st), "=&s"(m0s),   \
        "=&v"(wn), "=&s"(c0), "=&s"(c1), "=&s"(c2), "=&s"(c3), "=&s"(h0)
#define RC4_KSA_INS "v"(lanebase), "s"(sbase), "v"(ia), "s"(c16), "v"(d0)
#define KB(q) "v"(kb[q])
    /* the first identity rows as inputs: loop-invariant constants */
    uint32_t idc[RC4_KSA_IDREGS];
#pragma unroll
    for (int w = 0; w < RC4_KSA_IDREGS; w++) idc[w] = 0x03020100u + 0x04040404u * (uint32_t)w;
#define RC4_KSA_XIN RC4_KSA_IDIN
    if constexpr (NK == 16) {
        asm volatile(RC4_KSA_ASM_16
                     : RC4_KSA_OUTS
                     : RC4_KSA_INS, KB(0), KB(1), KB(2), KB(3), KB(4), KB(5), KB(6), KB(7), KB(8), KB(9), KB(10),
                       KB(11), KB(12), KB(13), KB(14), KB(15) RC4_KSA_XIN
                     : "vcc", "memory", "v60", "v61", "v62", "v63");
    } else {
        asm volatile(RC4_KSA_ASM_5
                     : RC4_KSA_OUTS
                     : RC4_KSA_INS, KB(0), KB(1), KB(2), KB(3), KB(4) RC4_KSA_XIN
                     : "vcc", "memory", "v60", "v61", "v62", "v63");
    }
#undef RC4_KSA_XIN
#undef KB
#undef RC4_KSA_INS
#undef RC4_KSA_OUTS
}

template <int NK>
DEVI void rc4_ksa_asm(uint32_t sbase, uint32_t lanebase, const uint32_t k[4]) {
    uint32_t kb[NK];
    rc4_kb_init<NK>(k, kb);
    rc4_ksa_asm_kb<NK>(sbase, lanebase, kb);
}

/* R2 (one KSA per candidate) runs the same rc4_ksa; its round-1 one-step-ahead KSA (S[j] and S[i+1] read
 * before the previous step's two stores, both repaired in registers) was 23 % slower once measured against
 * the grouped schedule (6.67 -> 8.20 G cand/s, round 2). */
/* PRGA bytes FROM..TO (1-based keystream positions), j carried in and out, XORed into d[] (LE-packed) */
template <int FROM, int TO>
DEVI void rc4_prga_span(uint8_t *S, uint32_t lanebase, uint32_t d[], uint32_t &j) {
#pragma unroll
    for (int i = FROM; i <= TO; i++) {
        const uint32_t ai = ((uint32_t)(i >> 2) << 8) + (uint32_t)(i & 3) + lanebase;
        const uint32_t si = lds_ld8(S, ai);
        j = j + si;
        const uint32_t aj = rc4_addr_sdwa(j, lanebase);
        const uint32_t sj = lds_ld8(S, aj);
        lds_st8(S, ai, sj);
        lds_st8(S, aj, si);
        const uint32_t ks = lds_ld8(S, rc4_addr_sdwa(si + sj, lanebase));
        d[(i - 1) >> 2] ^= ks << (8 * ((i - 1) & 3));
    }
}
template <int NB>
DEVI void rc4_prga(uint8_t *S, uint32_t lanebase, uint32_t d[]) {
    uint32_t j = 0;
#pragma unroll
    for (int i = 1; i <= NB; i++) {
        const uint32_t ai = ((uint32_t)(i >> 2) << 8) + (uint32_t)(i & 3) + lanebase;
        const uint32_t si = lds_ld8(S, ai);
        j = j + si;
        const uint32_t aj = rc4_addr_sdwa(j, lanebase);
        const uint32_t sj = lds_ld8(S, aj);
        lds_st8(S, ai, sj);
        lds_st8(S, aj, si);
        const uint32_t ks = lds_ld8(S, rc4_addr_sdwa(si + sj, lanebase));
        d[(i - 1) >> 2] ^= ks << (8 * ((i - 1) & 3));
    }
}

/* Two-byte PRGA for the early reject, with no stores: the box is re-initialised by the next KSA, so both
 * swaps live in registers and every read sees the post-KSA box, repaired where a swap touched its
 * position.  Reads: dword 0 (S[1], S[2]); S[j1]; S[t1] and S[j2] together; S[t2] -- four dependent LDS
 * round trips instead of six (read S[i], S[j], S[t] per byte, each after the previous byte's stores):
 * R3/R4 558.4 -> 559.6 M cand/s (round 2). */
template <>
DEVI void rc4_prga<2>(uint8_t *S, uint32_t lanebase, uint32_t d[]) {
    const uint32_t w0 = *(const uint32_t *)(S + lanebase);     /* S[0..3] after the KSA */
    const uint32_t s1 = (w0 >> 8) & 0xffu, s2o = (w0 >> 16) & 0xffu;
    /* byte 1: i = 1, j1 = S[1]; then S'[1] = S[j1], S'[j1] = s1 */
    const uint32_t j1 = s1;
    const uint32_t sj = lds_ld8(S, rc4_addr_sdwa(j1, lanebase));
    const uint32_t t1 = (s1 + sj) & 0xffu;
    /* byte 2: i = 2, s2 = S'[2], j2 = j1 + s2 */
    const uint32_t s2 = (j1 == 2u) ? s1 : s2o;
    const uint32_t j2 = (j1 + s2) & 0xffu;
    const uint32_t r1 = lds_ld8(S, rc4_addr_sdwa(t1, lanebase));
    const uint32_t rj = lds_ld8(S, rc4_addr_sdwa(j2, lanebase));
    const uint32_t k1 = (t1 == j1) ? s1 : ((t1 == 1u) ? sj : r1);           /* S'[t1] */
    const uint32_t sj2 = (j2 == j1) ? s1 : ((j2 == 1u) ? sj : rj);          /* S'[j2] */
    /* S''[2] = sj2, S''[j2] = s2 */
    const uint32_t t2 = (s2 + sj2) & 0xffu;
    const uint32_t r2 = lds_ld8(S, rc4_addr_sdwa(t2, lanebase));
    uint32_t k2 = (t2 == j1) ? s1 : ((t2 == 1u) ? sj : r2);                 /* S'[t2] */
    k2 = (t2 == 2u) ? sj2 : k2;
    k2 = (t2 == j2) ? s2 : k2;
    d[0] ^= k1 | (k2 << 8);
}

#endif

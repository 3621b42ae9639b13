/* RC4 schedule micro-benchmark for the PDF R3/R4 inner loop: 20 x (KSA-256 with a 16-byte key + 16-byte
 * PRGA) per lane, one 256-byte S-box per lane in LDS ([i/4][lane][i%4], one bank per lane).
 * Variants (all must produce identical per-lane output; checked against a CPU RC4):
 *   0  plain: S[j] read after the previous step's writes (one LDS round trip per step on the chain)
 *   1  one-step-ahead prefetch with register repairs (the production kernel's schedule)
 *   2  one-step-ahead, repairs as VGPR masks (no v_cmp -> SGPR -> v_cndmask hazard)
 *   3  grouped: S[4q..4q+3] read as one dword, S[i] writes kept in a register and stored once per group
 *   4  3 with the group loop rolled (instruction-fetch test)
 *   5  dword-prefetched s values, both swap stores per step (no register bookkeeping of the S[i] side)
 *   6  5 with the S[i] store deferred one step (the production schedule, dprf_kernels.hip rc4_ksa)
 *   7  6 with the next dword read two steps earlier (repairs against the last two steps)
 *  10-12 timing probes (not RC4): 9 without repairs / also without the group dword read / px repair only
 *   9  6 with the S[j] address in two instructions (SDWA byte-1 shift)
 *   8  6 with the S[i] repair applied lazily at the deferred store (first use of a read one step later)
 * Usage: rc4_bench [blocks_per_launch] [reps] */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>
#include "../dprf_amd/csrc/dev_crypto.h"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

DEVI uint32_t rc4_addr(uint32_t j, uint32_t lanebase) {
    return ((__builtin_amdgcn_ubfe(j, 2, 6)) << 8) | (j & 3u) | lanebase;
}
DEVI uint32_t rc4_addr_sdwa(uint32_t j, uint32_t lanebase) {
    uint32_t t = (j & 3u) | lanebase;
    asm("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
        : "+v"(t) : "v"(j));
    return t;
}
DEVI uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
DEVI uint32_t ld8(const uint8_t *b, uint32_t a) { return b[a]; }
DEVI void st8(uint8_t *b, uint32_t a, uint32_t v) { b[a] = (uint8_t)v; }
DEVI uint32_t posaddr(int i, uint32_t lanebase) { return ((uint32_t)(i >> 2) << 8) + (uint32_t)(i & 3) + lanebase; }
/* all-ones if a == b else 0, without a lane-mask SGPR */
DEVI uint32_t eqmask(uint32_t a, uint32_t b) { return umin32(a ^ b, 1u) - 1u; }
DEVI uint32_t sel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }

DEVI void sbox_init(uint8_t *S, uint32_t lanebase) {
#pragma unroll
    for (int w = 0; w < 64; w++) *(uint32_t *)(S + (w << 8) + lanebase) = 0x03020100u + 0x04040404u * (uint32_t)w;
}

template <int V>
DEVI void ksa(uint8_t *S, uint32_t lanebase, const uint32_t k[4]) {
    sbox_init(S, lanebase);
    uint32_t kb[16];
#pragma unroll
    for (int q = 0; q < 16; q++) kb[q] = (k[q >> 2] >> (8 * (q & 3))) & 0xffu;
    if (V == 0) {
        uint32_t j = 0;
#pragma unroll
        for (int i = 0; i < 256; i++) {
            const uint32_t si = ld8(S, posaddr(i, lanebase));
            j = (j + si + kb[i & 15]) & 0xffu;
            const uint32_t aj = rc4_addr(j, lanebase);
            const uint32_t sj = ld8(S, aj);
            st8(S, posaddr(i, lanebase), sj);
            st8(S, aj, si);
        }
    } else if (V == 1 || V == 2) {
        uint32_t j = 0, s_cur = 0, pj = 0, ps = 0, psj = 0;
#pragma unroll
        for (int i = 0; i < 256; i++) {
            const uint32_t ji = (j + s_cur + kb[i & 15]) & 0xffu;
            const uint32_t aj = rc4_addr(ji, lanebase);
            uint32_t x = ld8(S, aj);
            uint32_t y = 0;
            if (i < 255) y = ld8(S, posaddr(i + 1, lanebase));
            if (i > 0) {
                st8(S, posaddr(i - 1, lanebase), psj);
                st8(S, rc4_addr(pj, lanebase), ps);
                if (V == 1) x = (ji == pj) ? ps : ((ji == (uint32_t)(i - 1)) ? psj : x);
                else x = sel(eqmask(ji, pj), ps, sel(eqmask(ji, (uint32_t)(i - 1)), psj, x));
            }
            const uint32_t sj = x;
            if (i < 255) {
                uint32_t nxt = y;
                if (V == 1) {
                    if (i > 0) nxt = (pj == (uint32_t)(i + 1)) ? ps : nxt;
                    nxt = (ji == (uint32_t)(i + 1)) ? s_cur : nxt;
                } else {
                    if (i > 0) nxt = sel(eqmask(pj, (uint32_t)(i + 1)), ps, nxt);
                    nxt = sel(eqmask(ji, (uint32_t)(i + 1)), s_cur, nxt);
                }
                pj = ji; ps = s_cur; psj = sj; s_cur = nxt;
            } else {
                pj = ji; ps = s_cur; psj = sj;
            }
            j = ji;
        }
        st8(S, posaddr(255, lanebase), psj);
        st8(S, rc4_addr(pj, lanebase), ps);
    } else if (V == 4) {
        /* V3 with the group loop rolled (4 groups = 16 steps per iteration, so key bytes stay static):
         * ~1/16 of the code, to test whether V3's 30 KB of straight-line code is fetch-bound */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
        uint8_t *Sq = S + lanebase;
        uint32_t base = 0;
#pragma unroll 1
        for (int qq = 0; qq < 16; qq++) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                uint32_t s[4], m[4], x[4];
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                    for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                    s[r] = v;
                    j = j + v + kb[(4 * u + r) & 15];
                    m[r] = j & 0xffu;
                }
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t a = rc4_addr(m[r], lanebase);
                    x[r] = ld8(S, a);
                    st8(S, a, s[r]);
                }
                uint32_t Wn = 0;
                if (!(qq == 15 && u == 3)) Wn = *(const uint32_t *)(Sq + (u + 1) * 256);
                uint32_t Wf = W;
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t v = umin32(m[r] - base, 4u);
                    const uint32_t idr = 0x03020100u & ~(0xffu << (8 * r));
                    Wf = __builtin_amdgcn_perm(x[r], Wf, idr | (v << (8 * r)));
                    const uint32_t sh = (v << 3) & 31u;
                    Wf = __builtin_amdgcn_perm(s[r], Wf, 0x03020100u + ((4u - v) << sh));
                }
                *(uint32_t *)(Sq + u * 256) = Wf;
                W = Wn;
                base += 4u;
            }
            Sq += 1024;
        }
    } else if (V == 5) {
        /* Dword-prefetched s values, per-step stores: group q reads S[4q..4q+3] as one dword; s_r is byte
         * r unless an earlier step of the group swapped into it (S[j] = s with j = 4q+r).  Every step still
         * reads S[j] and writes S[i] = S[j], S[j] = s_i in program order, so LDS stays current for every
         * position and no in-group bookkeeping of the S[i] side is needed.  The j chain never waits on LDS
         * except for the one dword per four steps. */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[(4 * q + r) & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr(m[r], lanebase);
                const uint32_t x = ld8(S, a);
                st8(S, posaddr(4 * q + r, lanebase), x);
                st8(S, a, v);
            }
            if (q < 63) W = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
        }
    } else if (V == 6) {
        /* V5 with the S[i] = S[j] store deferred by one step, so the wave does not wait for the S[j] read
         * right after issuing it: step r+1's read precedes step r's S[i] store and is repaired when
         * j_{r+1} == i_r (it then must see x_r). */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
        uint32_t pi = 0, px = 0;            /* deferred store: position, value */
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = 4 * q + r;
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[i & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr(m[r], lanebase);
                uint32_t x = ld8(S, a);
                if (i > 0) {
                    st8(S, posaddr(i - 1, lanebase), px);
                    x = (m[r] == (uint32_t)(i - 1)) ? px : x;
                }
                st8(S, a, v);
                px = x;
            }
            if (q < 63) W = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
        }
        st8(S, posaddr(255, lanebase), px);
        (void)pi;
    } else if (V == 8) {
        /* V6 with the repair of x_i (j_i == i-1 -> the still-pending S[i-1]) applied lazily, right before x_i
         * is stored one step later: the wave's first use of a read is then after the next step's read, so the
         * wait covers a step of VALU work.  The asm statement pins that use after the read. */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
        uint32_t praw = 0, pflag = 0, pxf = 0;   /* x_{i-1} raw, (j_{i-1} == i-2), x_{i-2} final */
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = 4 * q + r;
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[i & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr(m[r], lanebase);
                const uint32_t x = ld8(S, a);
                if (i > 0) {
                    asm volatile("" : "+v"(praw) :: "memory");
                    const uint32_t xf = pflag ? pxf : praw;        /* x_{i-1} final */
                    st8(S, posaddr(i - 1, lanebase), xf);
                    pxf = xf;
                    pflag = m[r] == (uint32_t)(i - 1);
                }
                st8(S, a, v);
                praw = x;
            }
            if (q < 63) W = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
        }
        asm volatile("" : "+v"(praw) :: "memory");
        st8(S, posaddr(255, lanebase), pflag ? pxf : praw);
    } else if (V == 9) {
        /* V6 with the S[j] address built in two instructions: (j & 3) | lanebase, then byte 1 <- (j & 0xff) >> 2
         * by an SDWA shift that preserves the other bytes (rc4_addr: three instructions, two half-rate). */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
        uint32_t px = 0;
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = 4 * q + r;
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[i & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr_sdwa(j, lanebase);
                uint32_t x = ld8(S, a);
                if (i > 0) {
                    st8(S, posaddr(i - 1, lanebase), px);
                    x = (m[r] == (uint32_t)(i - 1)) ? px : x;
                }
                st8(S, a, v);
                px = x;
            }
            if (q < 63) W = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
        }
        st8(S, posaddr(255, lanebase), px);
    } else if (V == 10 || V == 11 || V == 12) {
        /* timing probes, NOT RC4 (results differ): 10 = variant 9 without any repair; 11 = 10 without the
         * per-group dword re-read (no LDS wait on the j chain); 12 = 9 with the px repair but no s repairs */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
        uint32_t px = 0;
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = 4 * q + r;
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
                s[r] = v;
                j = j + v + kb[i & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr_sdwa(j, lanebase);
                uint32_t x = ld8(S, a);
                if (i > 0) {
                    st8(S, posaddr(i - 1, lanebase), px);
                    if (V == 12) x = (m[r] == (uint32_t)(i - 1)) ? px : x;
                }
                st8(S, a, v);
                px = x;
            }
            (void)base; (void)s;
            if (V != 11) { if (q < 63) W = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase); }
            else W = W * 0x01010101u + px;
        }
        st8(S, posaddr(255, lanebase), px);
    } else if (V == 7) {
        /* V6 with the next group's dword read issued after step 1 of the current group: steps 2 and 3 may
         * still swap into the next group, so the next group's s values are also repaired against them. */
        uint32_t j = 0;
        uint32_t W = 0x03020100u, Wn = 0;
        uint32_t px = 0;
        uint32_t pm2 = 0xffffu, pm3 = 0xffffu, ps2 = 0, ps3 = 0;   /* previous group's steps 2, 3 */
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int i = 4 * q + r;
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
                if (q > 0) {
                    v = (pm2 == base + (uint32_t)r) ? ps2 : v;
                    v = (pm3 == base + (uint32_t)r) ? ps3 : v;
                }
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[i & 15];
                m[r] = j & 0xffu;
                const uint32_t a = rc4_addr(m[r], lanebase);
                uint32_t x = ld8(S, a);
                if (i > 0) {
                    st8(S, posaddr(i - 1, lanebase), px);
                    x = (m[r] == (uint32_t)(i - 1)) ? px : x;
                }
                st8(S, a, v);
                px = x;
                if (r == 1 && q < 63) Wn = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
            }
            pm2 = m[2]; pm3 = m[3]; ps2 = s[2]; ps3 = s[3];
            W = Wn;
        }
        st8(S, posaddr(255, lanebase), px);
    } else if (V == 3) {
        /* Grouped.  Group q covers positions 4q..4q+3 (one LDS dword of this lane).  Phase A (register only)
         * runs the j chain: s_r = value at position 4q+r before step r = the dword's byte r unless an
         * earlier step of the group swapped into it.  Then every step's S[j] is read and S[j] = s_r written
         * (in program order, so out-of-group positions are always current in LDS).  Phase B rebuilds the
         * group's dword with byte perms: byte r <- S[j_r] (from the dword itself when j_r is inside the
         * group, whose LDS copy is stale), and byte (j_r & 3) <- s_r when j_r is inside the group. */
        uint32_t j = 0;
        uint32_t W = 0x03020100u;
#pragma unroll
        for (int q = 0; q < 64; q++) {
            const uint32_t base = 4u * (uint32_t)q;
            uint32_t s[4], m[4], x[4];
#pragma unroll
            for (int r = 0; r < 4; r++) {
                uint32_t v = __builtin_amdgcn_ubfe(W, 8 * r, 8);
#pragma unroll
                for (int rr = 0; rr < r; rr++) v = (m[rr] == base + (uint32_t)r) ? s[rr] : v;
                s[r] = v;
                j = j + v + kb[(4 * q + r) & 15];
                m[r] = j & 0xffu;
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t a = rc4_addr(m[r], lanebase);
                x[r] = ld8(S, a);
                st8(S, a, s[r]);
            }
            uint32_t Wn = 0;
            if (q < 63) Wn = *(const uint32_t *)(S + ((q + 1) << 8) + lanebase);
            uint32_t Wf = W;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const uint32_t v = umin32(m[r] - base, 4u);     /* byte in group, 4 = outside */
                const uint32_t idr = 0x03020100u & ~(0xffu << (8 * r));
                Wf = __builtin_amdgcn_perm(x[r], Wf, idr | (v << (8 * r)));    /* byte r <- S[j_r] */
                const uint32_t sh = (v << 3) & 31u;
                Wf = __builtin_amdgcn_perm(s[r], Wf, 0x03020100u + ((4u - v) << sh)); /* byte v <- s_r */
            }
            *(uint32_t *)(S + (q << 8) + lanebase) = Wf;
            W = Wn;
        }
    }
}

DEVI void prga16(uint8_t *S, uint32_t lanebase, uint32_t d[4]) {
    uint32_t j = 0;
#pragma unroll
    for (int i = 1; i <= 16; i++) {
        const uint32_t ai = posaddr(i, lanebase);
        const uint32_t si = ld8(S, ai);
        j = j + si;
        const uint32_t aj = rc4_addr(j, lanebase);
        const uint32_t sj = ld8(S, aj);
        st8(S, ai, sj);
        st8(S, aj, si);
        const uint32_t ks = ld8(S, rc4_addr(si + sj, lanebase));
        d[(i - 1) >> 2] ^= ks << (8 * ((i - 1) & 3));
    }
}

__host__ __device__ inline uint32_t mix(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x;
}

template <int V>
__global__ void __launch_bounds__(64) k_rc4(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t S[16384];
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    const uint32_t lanebase = threadIdx.x << 2;
    uint32_t h[4] = {mix(g), mix(g + 0x9e3779b9u), mix(g ^ 0x5bd1e995u), mix(g * 3u + 1u)};
    uint32_t d[4] = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
    for (uint32_t x = 0; x < 20u; x++) {
        const uint32_t xx = x * 0x01010101u;
        uint32_t k[4] = {h[0] ^ xx, h[1] ^ xx, h[2] ^ xx, h[3] ^ xx};
        ksa<V>(S, lanebase, k);
        prga16(S, lanebase, d);
    }
    out[4 * g + 0] = d[0]; out[4 * g + 1] = d[1]; out[4 * g + 2] = d[2]; out[4 * g + 3] = d[3];
}

/* occupancy probe: variant 1 with WPB waves per workgroup; lane 0 of each wave records its CU and start/end time */
template <int WPB>
__global__ void __launch_bounds__(64 * WPB) k_rc4_occ(uint32_t *out, unsigned long long *rec) {
    __shared__ __attribute__((aligned(16))) uint8_t S[16384 * WPB];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t g = blockIdx.x * 64 * WPB + threadIdx.x;
    const uint32_t lanebase = (threadIdx.x & 63u) << 2;
    uint8_t *Sw = S + 16384 * (threadIdx.x >> 6);
    uint32_t h[4] = {mix(g), mix(g + 0x9e3779b9u), mix(g ^ 0x5bd1e995u), mix(g * 3u + 1u)};
    uint32_t d[4] = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
    for (uint32_t x = 0; x < 20u; x++) {
        const uint32_t xx = x * 0x01010101u;
        uint32_t k[4] = {h[0] ^ xx, h[1] ^ xx, h[2] ^ xx, h[3] ^ xx};
        ksa<1>(Sw, lanebase, k);
        prga16(Sw, lanebase, d);
    }
    out[4 * g + 0] = d[0]; out[4 * g + 1] = d[1]; out[4 * g + 2] = d[2]; out[4 * g + 3] = d[3];
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63u) == 0) {
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        const uint32_t w = g >> 6;
        rec[3 * w + 0] = ((unsigned long long)(xcc & 15u) << 32) | hw;
        rec[3 * w + 1] = t0;
        rec[3 * w + 2] = t1;
    }
}

static void occupancy(int blocks64, int wpb, uint32_t *dout) {
    const size_t waves = (size_t)blocks64;
    unsigned long long *drec;
    CHECK(hipMalloc(&drec, waves * 24));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, 0));
    if (wpb == 1) hipLaunchKernelGGL(k_rc4_occ<1>, dim3(blocks64), dim3(64), 0, 0, dout, drec);
    else hipLaunchKernelGGL(k_rc4_occ<2>, dim3(blocks64 / 2), dim3(128), 0, 0, dout, drec);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    std::vector<unsigned long long> rec(waves * 3);
    CHECK(hipMemcpy(rec.data(), drec, waves * 24, hipMemcpyDeviceToHost));
    /* per CU (xcc, se, sh, cu): max number of overlapping [t0, t1] */
    std::vector<std::vector<std::pair<unsigned long long, int>>> ev(8 * 16 * 2 * 16);
    for (size_t w = 0; w < waves; w++) {
        const unsigned long long id = rec[3 * w];
        const uint32_t hw = (uint32_t)id, xcc = (uint32_t)(id >> 32);
        const uint32_t cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
        const size_t key = ((xcc * 8 + se) * 2 + sh) * 16 + cu;
        ev[key].push_back({rec[3 * w + 1], +1});
        ev[key].push_back({rec[3 * w + 2], -1});
    }
    int ncu = 0, mx = 0; double mean = 0;
    for (auto &e : ev) {
        if (e.empty()) continue;
        std::sort(e.begin(), e.end(), [](auto &x, auto &y) { return x.first < y.first || (x.first == y.first && x.second < y.second); });
        int c = 0, m = 0;
        for (auto &p : e) { c += p.second; if (c > m) m = c; }
        ncu++; mean += m; if (m > mx) mx = m;
    }
    printf("occupancy probe wpb=%d: %.3f ms, %d CUs seen, max concurrent waves per CU: mean %.2f max %d -> %.1f M cand/s\n",
           wpb, ms, ncu, mean / ncu, mx, waves * 64 / ms / 1e3);
    CHECK(hipFree(drec));
}


/* co-scheduling probe: a pure-VALU kernel (52 MD5 compressions per lane, the R3/R4 key derivation's
 * work) on a second stream while the LDS-bound RC4 kernel runs */
__global__ void __launch_bounds__(256) k_md5x52(uint32_t *out) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    uint32_t h[4] = {mix(g), mix(g + 1u), mix(g + 2u), mix(g + 3u)};
    for (int i = 0; i < 52; i++) {
        uint32_t m[16] = {h[0], h[1], h[2], h[3], 0x80u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 128u, 0};
        md5_iv(h);
        md5_compress(h, m);
    }
    out[4 * g] = h[0] ^ h[1] ^ h[2] ^ h[3];
}

static void cosched(int blocks, uint32_t *dout, uint32_t *dout2) {
    hipStream_t sa, sb;
    CHECK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    const int mblocks = blocks / 4;   /* same number of lanes as the RC4 launch */
    float t[3];
    for (int mode = 0; mode < 3; mode++) {
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(a, 0));
        for (int r = 0; r < 3; r++) {
            if (mode != 1) hipLaunchKernelGGL(k_rc4<3>, dim3(blocks), dim3(64), 0, sa, dout);
            if (mode != 0) hipLaunchKernelGGL(k_md5x52, dim3(mblocks), dim3(256), 0, sb, dout2);
        }
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(b, 0));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&t[mode], a, b));
    }
    printf("co-scheduling: RC4 alone %.2f ms, MD5x52 alone %.2f ms, both on two streams %.2f ms (sum %.2f)\n",
           t[0] / 3, t[1] / 3, t[2] / 3, (t[0] + t[1]) / 3);
}

static void cpu_ref(uint32_t g, uint32_t d[4]) {
    uint32_t h[4] = {mix(g), mix(g + 0x9e3779b9u), mix(g ^ 0x5bd1e995u), mix(g * 3u + 1u)};
    d[0] = 0x11111111u; d[1] = 0x22222222u; d[2] = 0x33333333u; d[3] = 0x44444444u;
    for (uint32_t x = 0; x < 20u; x++) {
        uint8_t key[16], S[256];
        for (int q = 0; q < 16; q++) key[q] = (uint8_t)((h[q >> 2] >> (8 * (q & 3))) ^ x);
        for (int i = 0; i < 256; i++) S[i] = (uint8_t)i;
        uint32_t j = 0;
        for (int i = 0; i < 256; i++) { j = (j + S[i] + key[i & 15]) & 255; uint8_t t = S[i]; S[i] = S[j]; S[j] = t; }
        uint32_t i = 0; j = 0;
        for (int n = 0; n < 16; n++) {
            i = (i + 1) & 255; j = (j + S[i]) & 255; uint8_t t = S[i]; S[i] = S[j]; S[j] = t;
            d[n >> 2] ^= (uint32_t)S[(S[i] + S[j]) & 255] << (8 * (n & 3));
        }
    }
}

template <int V>
static double run(int blocks, int reps, uint32_t *dout, std::vector<uint32_t> &host) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_rc4<V>, dim3(blocks), dim3(64), 0, 0, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_rc4<V>, dim3(blocks), dim3(64), 0, 0, dout);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipMemcpy(host.data(), dout, host.size() * 4, hipMemcpyDeviceToHost));
    return ms / reps;
}


/* Round 2: two KSAs (passes 2x and 2x+1 of one candidate: their keystreams are independent, RC4(k,c) = c ^ ks)
 * interleaved step by step in one wave, variant-9 schedule each, S-boxes in two 16 KiB halves of a 32 KiB
 * block: 4 waves/CU instead of 9, but every wave carries two independent j chains (in-wave ILP instead of
 * cross-wave latency hiding). */
DEVI void ksa9x2(uint8_t *SA, uint8_t *SB, uint32_t lanebase, const uint32_t kA[4], const uint32_t kB[4]) {
    sbox_init(SA, lanebase);
    sbox_init(SB, lanebase);
    uint32_t kbA[16], kbB[16];
#pragma unroll
    for (int q = 0; q < 16; q++) {
        kbA[q] = (kA[q >> 2] >> (8 * (q & 3))) & 0xffu;
        kbB[q] = (kB[q >> 2] >> (8 * (q & 3))) & 0xffu;
    }
    uint32_t jA = 0, jB = 0, WA = 0x03020100u, WB = 0x03020100u, pxA = 0, pxB = 0;
#pragma unroll
    for (int q = 0; q < 64; q++) {
        const uint32_t base = 4u * (uint32_t)q;
        uint32_t sA[4], mA[4], sB[4], mB[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int i = 4 * q + r;
            uint32_t vA = __builtin_amdgcn_ubfe(WA, 8 * r, 8), vB = __builtin_amdgcn_ubfe(WB, 8 * r, 8);
#pragma unroll
            for (int rr = 0; rr < r; rr++) {
                vA = (mA[rr] == base + (uint32_t)r) ? sA[rr] : vA;
                vB = (mB[rr] == base + (uint32_t)r) ? sB[rr] : vB;
            }
            sA[r] = vA; sB[r] = vB;
            jA = jA + vA + kbA[i & 15]; jB = jB + vB + kbB[i & 15];
            mA[r] = jA & 0xffu; mB[r] = jB & 0xffu;
            const uint32_t aA = rc4_addr_sdwa(jA, lanebase), aB = rc4_addr_sdwa(jB, lanebase);
            uint32_t xA = ld8(SA, aA), xB = ld8(SB, aB);
            if (i > 0) {
                st8(SA, posaddr(i - 1, lanebase), pxA);
                st8(SB, posaddr(i - 1, lanebase), pxB);
                xA = (mA[r] == (uint32_t)(i - 1)) ? pxA : xA;
                xB = (mB[r] == (uint32_t)(i - 1)) ? pxB : xB;
            }
            st8(SA, aA, vA);
            st8(SB, aB, vB);
            pxA = xA; pxB = xB;
        }
        if (q < 63) {
            WA = *(const uint32_t *)(SA + ((q + 1) << 8) + lanebase);
            WB = *(const uint32_t *)(SB + ((q + 1) << 8) + lanebase);
        }
    }
    st8(SA, posaddr(255, lanebase), pxA);
    st8(SB, posaddr(255, lanebase), pxB);
}

__global__ void __launch_bounds__(64) k_rc4_x2(uint32_t *out) {
    __shared__ __attribute__((aligned(16))) uint8_t S[32768];
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;
    const uint32_t lanebase = threadIdx.x << 2;
    uint32_t h[4] = {mix(g), mix(g + 0x9e3779b9u), mix(g ^ 0x5bd1e995u), mix(g * 3u + 1u)};
    uint32_t d[4] = {0x11111111u, 0x22222222u, 0x33333333u, 0x44444444u};
    for (uint32_t x = 0; x < 20u; x += 2) {
        const uint32_t xa = x * 0x01010101u, xb = (x + 1) * 0x01010101u;
        uint32_t ka[4] = {h[0] ^ xa, h[1] ^ xa, h[2] ^ xa, h[3] ^ xa};
        uint32_t kb2[4] = {h[0] ^ xb, h[1] ^ xb, h[2] ^ xb, h[3] ^ xb};
        ksa9x2(S, S + 16384, lanebase, ka, kb2);
        prga16(S, lanebase, d);
        prga16(S + 16384, lanebase, d);
    }
    out[4 * g + 0] = d[0]; out[4 * g + 1] = d[1]; out[4 * g + 2] = d[2]; out[4 * g + 3] = d[3];
}

static double run_x2(int blocks, int reps, uint32_t *dout, std::vector<uint32_t> &host) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a)); CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(k_rc4_x2, dim3(blocks), dim3(64), 0, 0, dout);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a, 0));
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k_rc4_x2, dim3(blocks), dim3(64), 0, 0, dout);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipMemcpy(host.data(), dout, host.size() * 4, hipMemcpyDeviceToHost));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 65536;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t n = (size_t)blocks * 64;
    uint32_t *dout;
    CHECK(hipMalloc(&dout, n * 16));
    std::vector<uint32_t> ref(n * 4), got(n * 4);
    double ms[13];
    ms[0] = run<0>(blocks, reps, dout, ref);
    for (size_t g = 0; g < n; g += 9973) {
        uint32_t d[4];
        cpu_ref((uint32_t)g, d);
        if (memcmp(d, &ref[4 * g], 16)) { printf("variant 0 != CPU at lane %zu\n", g); return 1; }
    }
    int bad = 0;
#define VAR(V) ms[V] = run<V>(blocks, reps, dout, got); if (got != ref) { printf("variant %d MISMATCH\n", V); bad = 1; }
    VAR(1) VAR(2) VAR(3) VAR(4) VAR(5) VAR(6) VAR(7) VAR(8) VAR(9)
    ms[10] = run<10>(blocks, reps, dout, got); ms[11] = run<11>(blocks, reps, dout, got); ms[12] = run<12>(blocks, reps, dout, got);
    {
        const double mx2 = run_x2(blocks, reps, dout, got);
        if (got != ref) { printf("variant x2 MISMATCH\n"); bad = 1; }
        printf("variant x2 (two interleaved KSAs per wave, 32 KiB): %.3f ms -> %.1f M cand/s\n", mx2, n / mx2 / 1e3);
    }
    for (int v = 0; v < 13; v++)
        printf("variant %d: %.3f ms / launch of %zu lanes -> %.1f M cand/s (20 x KSA+PRGA16)\n", v, ms[v], n,
               n / ms[v] / 1e3);
    occupancy(blocks, 1, dout);
    occupancy(blocks, 2, dout);
    uint32_t *dout2;
    CHECK(hipMalloc(&dout2, n * 16));
    cosched(blocks, dout, dout2);
    return bad;
}

// valu_peak.hip -- measures gfx950 integer VALU issue rate for the instructions the verification kernels
// are made of (v_add3_u32, v_bitop3_b32, v_alignbit_b32, v_xor_b32, v_lshl_add_u64).  Each lane runs
// 8 independent dependency chains so issue, not latency, is the limit.  Prints lane-instructions/s.
//   hipcc --offload-arch=gfx950 -O3 tools/valu_peak.hip -o build/valu_peak && build/valu_peak
#include <hip/hip_runtime.h>
#include <cstdio>

#define ITERS 4096
#define CHAINS 8

/* round 4: does a wave64 VALU instruction cost less when a whole 32-lane half is inactive?  The add3 chain of OP 0 run
 * by lanes < 32 only (90), by the even lanes only (91), by lanes < 16 (92) */
template <int OP>
__global__ void __launch_bounds__(256) kmask(unsigned *out, unsigned seed) {
    const unsigned lane = threadIdx.x & 63u;
    const bool on = OP == 90 ? lane < 32u : OP == 91 ? (lane & 1u) == 0u : lane < 16u;
    if (!on) return;
    unsigned x[CHAINS];
    unsigned y = seed ^ threadIdx.x, z = seed * 3u + blockIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = seed + c * 77u + threadIdx.x;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) r ^= x[c];
    if (r == 0x12345678u) out[0] = r;
}

template <int OP>
__global__ void __launch_bounds__(256) k(unsigned *out, unsigned seed, int iters = ITERS) {
    unsigned x[CHAINS];
    unsigned y = seed ^ threadIdx.x, z = seed * 3u + blockIdx.x;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) x[c] = seed + c * 77u + threadIdx.x;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int c = 0; c < CHAINS; c++) {
            if (OP == 0) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 2) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
            if (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 5) asm volatile("v_xor_b32_e64 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 6) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 7) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 8) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 9) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 10) asm volatile("v_lshlrev_b32_e32 %0, 3, %0" : "+v"(x[c]));
            if (OP == 11) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                            asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y)); }
            if (OP == 12) asm volatile("v_alignbit_b32 %0, %1, %2, 27" : "=v"(x[c]) : "v"(x[c]), "v"(y));
            if (OP == 13) asm volatile("v_bfe_u32 %0, %0, 8, 8" : "+v"(x[c]));
            if (OP == 14) asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(x[c]) : "s"(seed));
            if (OP == 15) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 16) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 17) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 18) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 19) asm volatile("v_lshrrev_b32_e32 %0, 3, %0" : "+v"(x[c]));
            if (OP == 20) asm volatile("v_alignbyte_b32 %0, %0, %1, 1" : "+v"(x[c]) : "v"(y));
            if (OP == 21) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 22) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 23) asm volatile("v_sub_u32_e32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 24) asm volatile("v_not_b32_e32 %0, %0" : "+v"(x[c]));
            if (OP == 25) asm volatile("v_sad_u8 %0, %0, 0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 26) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 27) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 28) asm volatile("v_add_lshl_u32 %0, %0, %1, 2" : "+v"(x[c]) : "v"(y));
            if (OP == 29) asm volatile("v_lshlrev_b16_e32 %0, 3, %0" : "+v"(x[c]));
            if (OP == 30) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 31) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x[c]) : "v"(y));
            if (OP == 32) { /* independent VOP3 + VOP2 streams interleaved: even chains alignbit, odd chains xor */
                if (c & 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                else asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
            }
            if (OP == 33) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 34) asm volatile("v_ashrrev_i32_e32 %0, 3, %0" : "+v"(x[c]));
            if (OP == 35) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "=v"(x[c]) : "v"(x[c]));
            if (OP == 36) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc" : "+v"(x[c]) : "v"(y), "v"(z) : "vcc");
            if (OP == 37) { unsigned long long msk; asm volatile("v_cmp_eq_u32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %3, %1" : "+v"(x[c]), "=s"(msk) : "v"(y), "v"(z)); }
            if (OP == 38) asm volatile("v_cmp_eq_u32_e32 vcc, %0, %1" : : "v"(x[c]), "v"(y) : "vcc");
            if (OP == 39) { /* branch-free select: mask = ((a^b)-1) >>arith 31 ; x = ((z^x)&mask)^x */
                unsigned t;
                asm volatile("v_xor_b32 %1, %0, %2\n\tv_subrev_u32 %1, 1, %1\n\tv_ashrrev_i32 %1, 31, %1\n\tv_xor_b32 %1, %1, %0\n\tv_and_b32 %1, %1, %3\n\tv_xor_b32 %0, %0, %1" : "+v"(x[c]), "=&v"(t) : "v"(y), "v"(z));
            }
            if (OP == 40) { /* 64-bit add as a carry pair through VCC */
                asm volatile("v_add_co_u32_e32 %0, vcc, %0, %2\n\tv_addc_co_u32_e32 %1, vcc, %1, %3, vcc"
                             : "+v"(x[c]), "+v"(x[(c + 1) & (CHAINS - 1)]) : "v"(y), "v"(z) : "vcc");
            }
            if (OP == 41) { unsigned long long v = ((unsigned long long)x[c] << 32) | x[c];
                asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(v) : "v"(((unsigned long long)z << 32) | y));
                x[c] = (unsigned)v; }
            if (OP == 42) { unsigned long long v = ((unsigned long long)x[c] << 32) | y;
                asm volatile("v_lshrrev_b64 %0, 7, %0" : "+v"(v)); x[c] = (unsigned)v; }
            if (OP == 43) asm volatile("v_mov_b32_e32 %0, %1" : "=v"(x[c]) : "v"(x[(c + 3) & (CHAINS - 1)]));
            if (OP == 44) { /* 64-bit add as VOP3 carry pair with SGPR carry */
                unsigned long long cc;
                asm volatile("v_add_co_u32_e64 %0, %2, %0, %3\n\tv_addc_co_u32_e64 %1, %2, %1, %4, %2"
                             : "+v"(x[c]), "+v"(x[(c + 1) & (CHAINS - 1)]), "=&s"(cc) : "v"(y), "v"(z));
            }
            if (OP == 45) asm volatile("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:BYTE_0 src1_sel:DWORD" : : "v"(x[c]), "v"(y) : "vcc");
            if (OP == 46) { unsigned long long msk; asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(msk) : "v"(x[c]), "v"(y)); x[c] += (unsigned)msk; }
            if (OP == 47) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "s"((unsigned long long)z));
            if (OP == 48) { /* select through a VGPR mask: bfi(mask, a, b) */
                asm volatile("v_bfi_b32 %0, %1, %2, %0" : "+v"(x[c]) : "v"(y), "v"(z)); }
            if (OP == 49) asm volatile("v_min_u32_e32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 50) asm volatile("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:BYTE_0 src1_sel:DWORD\n\ts_nop 1\n\tv_cndmask_b32_e32 %0, %0, %2, vcc" : "+v"(x[c]) : "v"(y), "v"(z) : "vcc");
            if (OP == 51) asm volatile("v_lshrrev_b32_sdwa %0, 2, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0" : "+v"(x[c]) : "v"(y));
            if (OP == 52) asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "+v"(x[c]) : "v"(y));
            if (OP == 53) { /* the SHA-1 instruction mix of the ODF / Office KDF loops (round 4): per 8 instructions 3
                               alignbit, 2 add3, 2 bitop3, 1 xor -- 14.4 issue slots by the cost table of work.py */
                asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                             "v_alignbit_b32 %0, %0, %0, 2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t"
                             "v_add3_u32 %0, %0, %2, %1\n\tv_xor_b32 %0, %0, %1\n\t"
                             "v_alignbit_b32 %0, %0, %0, 31\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8"
                             : "+v"(x[c]) : "v"(y), "v"(z));
            }
            if (OP == 54) { /* the same eight as four interleaved pairs of the alignbit / add3 / bitop3 / xor streams */
                if (c & 1) asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\t"
                                        "v_xor_b32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 5" : "+v"(x[c]) : "v"(y), "v"(z));
                else asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                                  "v_alignbit_b32 %0, %0, %0, 2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x[c]) : "v"(y), "v"(z));
            }
            if (OP == 55) { /* the mix as separate statements: the compiler interleaves the eight chains */
                asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
                asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                asm volatile("v_alignbit_b32 %0, %0, %0, 2" : "+v"(x[c]));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
                asm volatile("v_add3_u32 %0, %0, %2, %1" : "+v"(x[c]) : "v"(y), "v"(z));
                asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                asm volatile("v_alignbit_b32 %0, %0, %0, 31" : "+v"(x[c]));
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x[c]) : "v"(y), "v"(z));
            }
            if (OP == 56) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 57) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 58) asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 59) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 60) { if (c & 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                            else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z)); }
            if (OP == 61) asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 62) asm volatile("v_xor_b32 %0, %0, %1\n\tv_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 63) asm volatile("v_add3_u32 %0, %0, %1, %2\n\tv_xor_b32_e64 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 64) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
            if (OP == 65) { if (c & 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                            else asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z)); }
            if (OP == 66) { if (c & 1) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
                            else asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z)); }
            if (OP == 67) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_bitop3_b32 %0, %0, %2, %1 bitop3:0xe8" : "+v"(x[c]) : "v"(y), "v"(z));
            if (OP == 68) { unsigned t = x[c]; /* bitop3 with 16 independent chains (two per x) */
                asm volatile("v_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %3, %2 bitop3:0x96" : "+v"(x[c]), "+v"(t) : "v"(y), "v"(z));
                x[c] ^= t; }
            /* half-rate (add3) / full-rate (xor) patterns over the eight independent chains (round 4) */
            if (OP == 70) { if ((c >> 1) & 1) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                            else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z)); }   /* HHFFHHFF */
            if (OP == 71) { if (c >= 4) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                            else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z)); }   /* HHHHFFFF */
            if (OP == 72) { if (c == 7) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y));
                            else asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z)); }   /* 7H 1F */
            if (OP == 73) { if (c == 7) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                            else asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y)); }               /* 7F 1H */
            if (OP == 74) { if (c & 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
                            else asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c])); }                /* H F (bitop3) */
            /* round 4: the ODF KDF loop's instruction counts per 2 PBKDF2 iterations (887 alignbit, 566 add3, 516 bitop3,
             * 268 xor, 110 add) as a 21-instruction pattern per chain, and the same work with every add3 as two v_add
             * (26 instructions, 30 % half-rate instead of 62 %) */
            if (OP == 80) {
                asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\t"
                             "v_add3_u32 %0, %0, %1, %2\n\tv_alignbit_b32 %0, %0, %0, 2\n\tv_add3_u32 %0, %0, %2, %1\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_alignbit_b32 %0, %0, %0, 31\n\t"
                             "v_xor_b32 %0, %0, %1\n\tv_add3_u32 %0, %0, %1, %2\n\tv_alignbit_b32 %0, %0, %0, 5\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8\n\tv_add3_u32 %0, %0, %2, %1\n\t"
                             "v_alignbit_b32 %0, %0, %0, 30\n\tv_add_u32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 1\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_add3_u32 %0, %0, %1, %2\n\t"
                             "v_alignbit_b32 %0, %0, %0, 27\n\tv_xor_b32 %0, %0, %2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\t"
                             "v_alignbit_b32 %0, %0, %0, 2" : "+v"(x[c]) : "v"(y), "v"(z));
            }
            if (OP == 81) {
                asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\t"
                             "v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\tv_alignbit_b32 %0, %0, %0, 2\n\t"
                             "v_add_u32 %0, %0, %2\n\tv_add_u32 %0, %0, %1\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_alignbit_b32 %0, %0, %0, 31\n\t"
                             "v_xor_b32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\tv_alignbit_b32 %0, %0, %0, 5\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8\n\tv_add_u32 %0, %0, %2\n\tv_add_u32 %0, %0, %1\n\t"
                             "v_alignbit_b32 %0, %0, %0, 30\n\tv_add_u32 %0, %0, %1\n\tv_alignbit_b32 %0, %0, %0, 1\n\t"
                             "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %2\n\t"
                             "v_alignbit_b32 %0, %0, %0, 27\n\tv_xor_b32 %0, %0, %2\n\tv_bitop3_b32 %0, %0, %1, %2 bitop3:0xca\n\t"
                             "v_alignbit_b32 %0, %0, %0, 2" : "+v"(x[c]) : "v"(y), "v"(z));
            }
            if (OP == 82) { /* the 21-instruction ODF pattern as separate statements: the compiler interleaves the chains */
                asm("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
                asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 2" : "+v"(x[c]));
                asm("v_add3_u32 %0, %0, %2, %1" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 31" : "+v"(x[c]));
                asm("v_xor_b32 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 5" : "+v"(x[c]));
                asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_add3_u32 %0, %0, %2, %1" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 30" : "+v"(x[c]));
                asm("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 1" : "+v"(x[c]));
                asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x[c]));
                asm("v_xor_b32 %0, %0, %2" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(x[c]) : "v"(y), "v"(z));
                asm("v_alignbit_b32 %0, %0, %0, 2" : "+v"(x[c]));
            }
            if (OP == 83) { /* round 5: the 21-instruction ODF pattern on two chains in instruction-level lockstep (A, B, A, B,
                               ...): every instruction is followed by the same one on the other chain, independent of it */
                if ((c & 1) == 0)
                    asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_alignbit_b32 %1, %1, %1, 27\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0xca\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0xca\n\tv_add3_u32 %0, %0, %2, %3\n\tv_add3_u32 %1, %1, %2, %3\n\tv_alignbit_b32 %0, %0, %0, 2\n\tv_alignbit_b32 %1, %1, %1, 2\n\tv_add3_u32 %0, %0, %3, %2\n\tv_add3_u32 %1, %1, %3, %2\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n\tv_alignbit_b32 %0, %0, %0, 31\n\tv_alignbit_b32 %1, %1, %1, 31\n\tv_xor_b32 %0, %0, %2\n\tv_xor_b32 %1, %1, %2\n\tv_add3_u32 %0, %0, %2, %3\n\tv_add3_u32 %1, %1, %2, %3\n\tv_alignbit_b32 %0, %0, %0, 5\n\tv_alignbit_b32 %1, %1, %1, 5\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0xe8\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0xe8\n\tv_add3_u32 %0, %0, %3, %2\n\tv_add3_u32 %1, %1, %3, %2\n\tv_alignbit_b32 %0, %0, %0, 30\n\tv_alignbit_b32 %1, %1, %1, 30\n\tv_add_u32 %0, %0, %2\n\tv_add_u32 %1, %1, %2\n\tv_alignbit_b32 %0, %0, %0, 1\n\tv_alignbit_b32 %1, %1, %1, 1\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0x96\n\tv_add3_u32 %0, %0, %2, %3\n\tv_add3_u32 %1, %1, %2, %3\n\tv_alignbit_b32 %0, %0, %0, 27\n\tv_alignbit_b32 %1, %1, %1, 27\n\tv_xor_b32 %0, %0, %3\n\tv_xor_b32 %1, %1, %3\n\tv_bitop3_b32 %0, %0, %2, %3 bitop3:0xca\n\tv_bitop3_b32 %1, %1, %2, %3 bitop3:0xca\n\tv_alignbit_b32 %0, %0, %0, 2\n\tv_alignbit_b32 %1, %1, %1, 2" : "+v"(x[c]), "+v"(x[c + 1]) : "v"(y), "v"(z));
            }
            if (OP == 4) {
                unsigned long long v = ((unsigned long long)x[c] << 32) | y;
                asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(v) : "v"(((unsigned long long)z << 32) | z));
                x[c] = (unsigned)v ^ (unsigned)(v >> 32);
            }
        }
    }
    unsigned r = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; c++) r ^= x[c];
    if (r == 0x12345678u) out[0] = r;
}

template <int OP>
double run_mask(const char *name, int blocks, double lanes_on) {
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(kmask<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(kmask<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    /* wave-instructions per second, whatever the active lanes: the cost of an instruction with a partial EXEC */
    const double wave_instr = (double)reps * blocks * 4.0 * ITERS * CHAINS;
    printf("%-28s %.3f ms  %.2f G wave-instr/s  (active-lane instr %.2f T/s)\n", name, ms / reps,
           wave_instr / (ms / 1e3) / 1e9, wave_instr * lanes_on / (ms / 1e3) / 1e12);
    (void)hipFree(d);
    return ms;
}

template <int OP>
double run(const char *name, int blocks, int per_iter) {
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u, ITERS);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    const int reps = 5;
    for (int r = 0; r < reps; r++) hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u + r, ITERS);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    double lane_instr = (double)reps * blocks * 256.0 * ITERS * CHAINS * per_iter;
    double rate = lane_instr / (ms / 1e3);
    printf("%-16s blocks=%6d  %.2f T lane-instr/s  (%.1f%% of 256x4x32x2.4GHz = 78.64T)\n", name, blocks, rate / 1e12,
           100.0 * rate / 78.6432e12);
    (void)hipFree(d);
    return rate;
}

/* round 5: the issue rate by waves per SIMD.  One generation of `wps` 256-thread blocks per CU (4 waves: one per SIMD),
 * each wave running `iters` iterations of the pattern, best of 3 launches after a warm-up; the rate is per SIMD against
 * its full-rate peak (2 cycles per wave64 instruction at 2.4 GHz), so 100 % = one full-rate instruction every 2 cycles */
template <int OP>
void run_occ(const char *name, int per_iter, int iters) {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *d;
    (void)hipMalloc(&d, 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL(k<OP>, dim3(ncu * 8), dim3(256), 0, 0, d, 1u, iters);
    (void)hipDeviceSynchronize();
    printf("%-22s", name);
    for (int wps : {1, 2, 3, 4, 6, 8}) {
        const int blocks = ncu * wps;
        float best = 1e30f;
        for (int r = 0; r < 3; r++) {
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 2u + r, iters);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            best = ms < best ? ms : best;
        }
        const double lane_instr = (double)blocks * 256.0 * iters * CHAINS * per_iter;
        const double rate = lane_instr / (best / 1e3);
        /* cycles per wave-instruction on a SIMD: (SIMD-cycles) / (wave-instructions per SIMD) */
        const double cyc = best / 1e3 * 2.4e9 / ((double)wps * iters * CHAINS * per_iter);
        printf("  w%d %5.1f%% %4.2fc", wps, 100.0 * rate / 78.6432e12, cyc);
    }
    printf("\n");
    (void)hipFree(d);
}

int main(int argc, char **argv) {
    const int blocks = 32768;
    if (argc > 1 && argv[1][0] == 'o') {   /* "occ": issue rate by waves per SIMD */
        const int it = 8192;
        run_occ<3>("xor (F)", 1, it);
        run_occ<65>("bitop3|xor indep (F)", 1, it);
        run_occ<68>("bitop3 16 chains (F)", 2, it);
        run_occ<2>("alignbit (H)", 1, it);
        run_occ<0>("add3 (H)", 1, it);
        run_occ<74>("alignbit|bitop3 alt", 1, it);
        run_occ<70>("HHFF", 1, it);
        run_occ<73>("7F 1H", 1, it);
        run_occ<80>("odf mix (21)", 21, it / 8);
        run_occ<82>("odf mix (21) il", 21, it / 8);
        run_occ<83>("odf mix (21) lockstep2", 21, it / 8);
        return 0;
    }
    if (argc > 1) {   /* "mix": the KDF instruction mix against the additive slot model (78.64 T x 8 / 14.4) */
        run<53>("sha1 mix x8", blocks, 8);
        run<54>("sha1 mix x4 il", blocks, 4);
        run<55>("sha1 mix stmts", blocks, 8);
        run<56>("alignbit+add3", blocks, 2);
        run<57>("alignbit+bitop3", blocks, 2);
        run<58>("add3+xor", blocks, 2);
        run<59>("bitop3+xor", blocks, 2);
        run<60>("add3|xor indep", blocks, 1);
        run<61>("add3>add dep", blocks, 2);
        run<62>("xor>add3 dep", blocks, 2);
        run<63>("add3>xor_e64 dep", blocks, 2);
        run<64>("alignbit>xor dep", blocks, 2);
        run<65>("bitop3|xor indep", blocks, 1);
        run<66>("alignbit|bitop3 indep", blocks, 1);
        run<67>("bitop3>bitop3 dep", blocks, 2);
        run<70>("HHFF x2 indep", blocks, 1);
        run<71>("HHHHFFFF indep", blocks, 1);
        run<72>("7H 1F indep", blocks, 1);
        run<73>("7F 1H indep", blocks, 1);
        run<74>("alignbit|bitop3 alt", blocks, 1);
        run<80>("odf mix (21, add3)", blocks, 21);
        run<81>("odf mix (26, add3 as 2 add)", blocks, 26);
        run<82>("odf mix (21) chains interleaved", blocks, 21);
        run<83>("odf mix (21) 2-chain lockstep", blocks, 21);
        printf("per 21-instruction unit of work: cycles = 21 x 157.29 T / rate(80) vs 26 x 157.29 T / rate(81)\n");
        run<2>("v_alignbit_b32", blocks, 1);
        run<0>("v_add3_u32", blocks, 1);
        run<1>("v_bitop3_b32", blocks, 1);
        run_mask<90>("add3, lanes 0-31 only", blocks, 32);
        run_mask<91>("add3, even lanes only", blocks, 32);
        run_mask<92>("add3, lanes 0-15 only", blocks, 16);
        printf("(all 64 lanes: v_add3_u32 above, lane-instr/s / 64 = wave-instr/s)\n");
        printf("slot model for the mix: %.2f T lane-instr/s\n", 78.6432 * 8 / 14.4);
        return 0;
    }
    run<3>("v_xor_b32", blocks, 1);
    run<31>("v_cndmask vcc", blocks, 1);
    run<47>("v_cndmask e64 s", blocks, 1);
    run<38>("v_cmp_eq e32", blocks, 1);
    run<45>("v_cmp_eq sdwa", blocks, 1);
    run<46>("v_cmp_eq e64+add", blocks, 2);
    run<36>("cmp+cndmask vcc", blocks, 2);
    run<37>("cmp+cndmask e64", blocks, 2);
    run<50>("cmp_sdwa+nop+cnd", blocks, 2);
    run<39>("xor-mask select", blocks, 6);
    run<48>("v_bfi_b32", blocks, 1);
    run<51>("lshr sdwa byte1", blocks, 1);
    run<52>("add sdwa byte0", blocks, 1);
    run<49>("v_min_u32", blocks, 1);
    run<40>("add_co+addc (vcc) pair", blocks, 2);
    run<44>("add_co+addc e64 pair", blocks, 2);
    run<41>("v_lshl_add_u64", blocks, 1);
    run<42>("v_lshrrev_b64", blocks, 1);
    run<43>("v_mov_b32", blocks, 1);
    return 0;
}

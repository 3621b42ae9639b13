#!/usr/bin/env python3
"""Generate dprf_amd/csrc/rc4_ksa_asm.h: the RC4 key schedule of the PDF R2-R4 kernels as one gfx950 inline-asm
block per key length (pdf_password_verifier.c:157-176 via EVP_rc4; RC4 itself: S = identity, then for i = 0..255
j += S[i] + K[i % n]; swap(S[i], S[j])).

Why asm: the compiled C++ schedule (rc4_dev.h rc4_ksa) issues 16-17 VALU instructions per group of two steps
(~31 issue slots: byte extracts, compare + select pairs, a u16 merge in two steps); the same dataflow fits in 12,
with the byte selects folded into SDWA operands -- and only asm keeps LLVM from re-materialising or re-ordering
them.  What bounds this loop on gfx950 is the length of each wave's instruction stream and its LDS round trip (9
chains per CU): every variant that added instructions or LDS operations lost, every one that
removed some won.  The schedule is rc4_ksa's group-deferred one (rc4_dev.h): per group q (i0 = 2q, i1 = 2q + 1)

    wait for W = S[i0] | S[i1] << 8            (read at the end of group q - 1; lgkmcnt(1): the u16 store
                                                 issued after it may stay in flight -- LDS completes in order)
    j += W + K[i0]                              (only j's low byte is ever used: W's byte 1 above it is harmless)
    a0 = (j & 3) | lanebase (v_bitop3); a0.byte1 = j.byte0 >> 2  -> address of S[j] in the [i/4][lane][i%4] layout
    hit1 = (j.byte0 == i1)                      (i1 an inline constant while <= 64, else byte 1 of a VGPR (i0, i1)
                                                 bumped by 0x0202 once per group: no SALU in the loop)
    x0 = S[j]; S[j] = W.byte0
    v1 = hit1 ? W.byte0 : W.byte1               (one SDWA cndmask: the current S[i1])
    j += v1 + K[i1];  a1 likewise;  hit0 = (j.byte0 == i0)
    x1 = S[j]; S[j] = v1
    W = S[i0 + 2] | S[i0 + 3] << 8              (after both S[j] stores, before the deferred S[i] stores)
    wait for x0, x1 (lgkmcnt(1))
    m = hit0 ? v1 : x0;  m.byte1 = hit0 ? x0 : x1                -> S[i0], S[i1] as one u16
    store m at S[i0]

The identity is written by 64 ds_write_addtid_b32, rows 0..23 straight from 24 loop-invariant input VGPRs (rc4_dev.h
idc[]) and the rest from an add chain.  Hazards: every VCC consumer (v_cndmask) is at least two instructions after
the v_cmp that writes VCC (the LDS instructions in between count as wait states); the first ds_write_addtid after
the M0 write is one instruction behind it (tests/test_rc4_asm.py lds_hazards).  The block ends with lgkmcnt(0), so
the compiler never sees an LDS operation of this block in flight.
Requirements (checked by the caller): the S-box area starts at an LDS address whose low 16 bits are zero (the
SDWA byte-1 insert overwrites bits 8-15 of lanebase) and lanebase = area + 4 * lane.

The schedules measured and rejected in rounds 3-5 (early reads, late merges, prefetch, SALU compare constants, the
j counter, the b128 identity, d16 merges, split adds, v_and_or addresses, ds_mskor, byte pairs) are listed with their
numbers in HISTORY.md; this generator emits only the shipped one.

Usage: tools/gen_rc4_ksa_asm.py > dprf_amd/csrc/rc4_ksa_asm.h
       tools/gen_rc4_ksa_asm.py --no-m0-wait   (test input only: round 4's first identity schedule, which stored row 0
                                                right behind the M0 write and lost it on the MI355X -- the hazard model
                                                of tests/test_rc4_asm.py must reject it)
"""

KEYLENS = (5, 16)   # R2 / R3-R4 with 40-bit keys use 5 bytes, R3/R4 128-bit keys 16 (EVP_rc4 reads 16)
IDREGS = 24         # identity rows 0..23 as input VGPRs (round 5: R3/R4 625.5 vs 623.1 M, profiles/ab_r24_r05b.txt)
FIRST_IC = 32       # first group whose i1 is past the inline constants (0..64): compares read the (i0, i1) VGPR


def pos(i):
    """byte offset of S[i] from the lane's column base"""
    return ((i >> 2) << 8) + (i & 3)


def ksa(nk, m0_wait=True):
    # operands: %0 j, %1 W, %2 x0, %3 x1, %4 v1, %5 a0, %6 a1, %7 m, %8 (SGPR, unused), %9 m0save (SGPR), %10 (i0, i1),
    #           %11-%15 (SGPR pairs, unused), %16 lanebase, %17 sbase (SGPR, the area's LDS address for
    #           ds_write_addtid), %18-%20 (unused inputs), %21.. key bytes, then the identity rows.  The unused operands
    #           keep the register assignment of the measured build (rc4_dev.h rc4_ksa_asm_kb).
    J, W, X0, X1, V1, A0, A1, M, _, M0S, IC = ("%%%d" % k for k in range(11))
    LB, SB = "%16", "%17"
    KB = ["%%%d" % (21 + k) for k in range(nk)]
    out = []
    e = out.append
    identity(e, M, M0S, SB, ["%%%d" % (21 + nk + k) for k in range(IDREGS)], m0_wait)
    e("v_mov_b32 %s, 0" % J)
    e("v_mov_b32 %s, 0x100" % W)         # group 0 = S[0] | S[1] << 8 of the identity
    i0f = 2 * FIRST_IC
    e("v_mov_b32 %s, 0x%x" % (IC, i0f | ((i0f + 1) << 8)))

    def cmp(i, q, sel):
        if q < FIRST_IC:
            e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, sel))

    for q in range(128):
        i0, i1 = 2 * q, 2 * q + 1
        if q > 0:
            e("s_waitcnt lgkmcnt(1)")
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, W, KB[i0 % nk]))
        e(addr_lo(A0, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        cmp(i1, q, "BYTE_1")
        e("ds_read_u8 %s, %s" % (X0, A0))
        e("ds_write_b8 %s, %s" % (A0, W))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_0"
          % (V1, W, W))
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nk]))
        e(addr_lo(A1, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        cmp(i0, q, "BYTE_0")
        e("ds_read_u8 %s, %s" % (X1, A1))
        e("ds_write_b8 %s, %s" % (A1, V1))
        if FIRST_IC <= q < 127:
            e("v_add_u32 %s, 0x202, %s" % (IC, IC))
        if q < 127:
            e("ds_read_u16 %s, %s offset:%d" % (W, LB, pos(i0 + 2)))
            e("s_waitcnt lgkmcnt(1)")
        else:
            e("s_waitcnt lgkmcnt(0)")
        # the deferred S[i0], S[i1] of group q as one u16 (VCC = hit0)
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "
          "src1_sel:DWORD" % (M, X1, X0))
        e("ds_write_b16 %s, %s offset:%d" % (LB, M, pos(2 * q)))
    e("s_waitcnt lgkmcnt(0)")
    return out


def addr_lo(A, J, LB):
    """A = (j & 3) | lanebase as v_bitop3_b32 (LUT 0xea = (s0 & s1) | s2), which issues at full rate on gfx950 unless its
    three sources share a VGPR bank (profiles/vgpr_bank_r04.txt), where v_and_or_b32 is half rate (round 4: R3/R4
    625.7 -> 628.3 M, profiles/ab_r24_b3addr_r04n.txt)"""
    return "v_bitop3_b32 %s, %s, 3, %s bitop3:0xea" % (A, J, LB)


def identity(e, M, M0S, SB, ids, m0_wait=True):
    """S = identity: dword w of lane l at area + 256 w + 4 l; ids: input VGPRs holding rows 0..len(ids)-1 (loop-invariant
    constants the kernel keeps in registers), so only the rows after them need the add chain"""
    e("s_mov_b32 %s, m0" % M0S)
    e("s_mov_b32 m0, %s" % SB)
    n = len(ids)
    # the v_mov is also the wait state an M0 write needs before an LDS instruction that reads M0 (ds_write_addtid)
    mov = "v_mov_b32 %s, 0x%x" % (M, (0x03020100 + 0x04040404 * n) & 0xffffffff)
    if m0_wait:
        e(mov)
    for w in range(n):
        e("ds_write_addtid_b32 %s offset:%d" % (ids[w], 256 * w))
    if not m0_wait:
        e(mov)
    for w in range(n, 64):
        e("ds_write_addtid_b32 %s offset:%d" % (M, 256 * w))
        if w < 63:
            e("v_add_u32 %s, 0x4040404, %s" % (M, M))
    e("s_mov_b32 m0, %s" % M0S)


def main():
    import sys
    m0_wait = "--no-m0-wait" not in sys.argv
    print("/* rc4_ksa_asm.h -- GENERATED by tools/gen_rc4_ksa_asm.py (see there for the schedule); do not edit. */")
    print("#ifndef DPRF_RC4_KSA_ASM_H")
    print("#define DPRF_RC4_KSA_ASM_H")
    print("#define RC4_KSA_IDREGS %d   /* identity rows 0..%d as input VGPRs after the keys (rc4_dev.h idc[]) */"
          % (IDREGS, IDREGS - 1))
    print("#define RC4_KSA_IDIN " + "".join(', "v"(idc[%d])' % k for k in range(IDREGS)))
    for nk in KEYLENS:
        print("#define RC4_KSA_ASM_%d \\" % nk)
        for ln in ksa(nk, m0_wait):
            print('    "%s\\n\\t" \\' % ln)
        print('    ""')
    print("#endif")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Generate dprf_amd/csrc/rc4_ksa_asm.h: the RC4 key schedule of the PDF R2-R4 kernels as one gfx950 inline-asm
block per key length (pdf_password_verifier.c:157-176 via EVP_rc4; RC4 itself: S = identity, then for i = 0..255
j += S[i] + K[i % n]; swap(S[i], S[j])).

Why asm: the compiled C++ schedule (rc4_dev.h rc4_ksa) issues 16-17 VALU instructions per group of two steps
(~31 issue slots: byte extracts, compare + select pairs, a u16 merge in two steps); the same dataflow fits in 12,
with the byte selects folded into SDWA operands -- and only asm keeps LLVM from re-materialising or re-ordering
them.  What bounds this loop on gfx950 is the length of each wave's instruction stream (LdsUtil 0.5, VALU not
saturated, 9 waves per CU): every variant that added instructions lost, every one that removed some won, so the
schedule minimises instructions per group (20; 19 while the compare constants are inline), SALU included --
except that LDS time counts too: 16 ds_write_b128 for the identity instead of 64 ds_write_addtid_b32 (48 instead
of 131 instructions per KSA) lost 3 %.  The schedule is rc4_ksa's group-deferred one
(rc4_dev.h): per group q (i0 = 2q, i1 = 2q + 1)

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

The identity is written by 64 ds_write_addtid_b32 (identity; identity_b128 measured slower).  Hazards: every VCC consumer (v_cndmask) is at
least two instructions after the v_cmp that writes VCC (the LDS instructions in between count as wait states).
The block ends with lgkmcnt(0), so the compiler never sees an LDS operation of this block in flight.
Requirements (checked by the caller): the S-box area starts at an LDS address whose low 16 bits are zero (the
SDWA byte-1 insert overwrites bits 8-15 of lanebase) and lanebase = area + 4 * lane.

Usage: tools/gen_rc4_ksa_asm.py > dprf_amd/csrc/rc4_ksa_asm.h
       tools/gen_rc4_ksa_asm.py --early-read > <variant header>   (A/B: each S[j] read one instruction earlier)
       tools/gen_rc4_ksa_asm.py --late-merge > <variant header>   (A/B: group q-1's S[i] merge + store issued
                                                                    inside group q, between a0 and the S[j] read)
       tools/gen_rc4_ksa_asm.py --prefetch > <variant header>     (A/B: the next pair read at the start of each
                                                                    group and repaired for its S[j] stores)
       tools/gen_rc4_ksa_asm.py --salu-consts > <variant header>  (A/B, round-3 first version: compare constants
                                                                    through two s_movk per group)
       tools/gen_rc4_ksa_asm.py --early-v1 > <variant header>     (A/B: step 1's compare-select and j add hoisted
                                                                    above step 0's LDS pair, same instructions)
       tools/gen_rc4_ksa_asm.py --jctr > <variant header>         (A/B: i0 / i1 counted in byte 3 of j, key registers
                                                                    carrying the counter steps: 603 vs 612 M, slower)
       tools/gen_rc4_ksa_asm.py --ic4 / --d16merge > <variant header>  (round 4 A/B: (i0, i1) of two groups in one
                                                                    register, one v_add per two groups / x0, x1 by
                                                                    d16 loads into one register, merged by one v_perm)
       tools/gen_rc4_ksa_asm.py --and-or > <variant header>        (the S[j] address's low byte by v_and_or_b32, half
                                                                    rate, as before round 4; default: v_bitop3_b32)
       tools/gen_rc4_ksa_asm.py --mskor > <variant header>          (round 5 A/B: S[j] read + store as one
                                                                    ds_mskor_rtn_b32: 4 LDS ops per group, 18 VALU)
       tools/gen_rc4_ksa_asm.py --bytes > <variant header>          (round 5 A/B: the S[i] pair as two byte loads /
                                                                    stores, full-rate selects: 36 VALU cycles per
                                                                    group instead of 40, 8 LDS ops instead of 6)
       tools/gen_rc4_ksa_asm.py --idregs 24 [--no-m0-wait] > <hdr>  (round 4 A/B: identity rows 0-23 from input VGPRs;
                                                                    --no-m0-wait: round 4's first, wrong, schedule)
       tools/gen_rc4_ksa_asm.py --b128-identity > <variant header>  (A/B: the identity as 16 ds_write_b128 + 30
                                                                    64-bit adds: 612 -> 595 M, the b128 stores cost
                                                                    more LDS time than the instructions they save)
"""

KEYLENS = (5, 16)   # R2 / R3-R4 with 40-bit keys use 5 bytes, R3/R4 128-bit keys 16 (EVP_rc4 reads 16)


def pos(i):
    """byte offset of S[i] from the lane's column base"""
    return ((i >> 2) << 8) + (i & 3)


def nkr_of(nk, jctr):
    """key registers the block reads: with the j counter every register must serve one step parity, so the 5-byte
    key is passed as 10 registers (key byte i % 5 with the counter step of i's parity)"""
    return 10 if (jctr and nk % 2) else nk


def ksa(nk, early_read=False, late_merge=False, prefetch=False, vconst=False, b128=False, jctr=False, ic4=False,
        d16=False, split=False, b3addr=False, idregs=0, m0_wait=True):
    # operands: %0 j, %1 W, %2 x0, %3 x1, %4 v1, %5 a0, %6 a1, %7 m, %8 stmp (SGPR), %9 m0save (SGPR), %10 Wn / IC,
    #           %11-%15 SGPR pairs (prefetch repairs: j0 == p2, j0 == p3, j1 == p2, j1 == p3; hit0),
    #           %16 lanebase, %17 sbase (SGPR, the area's LDS address for ds_write_addtid), %18 identity address
    #           (VGPR), %19 0x1010101010101010 (SGPR pair), %20 first identity dword of the lane, %21.. key bytes;
    #           the b128 identity's data quad is the clobbered v[60:63] (a register tuple operand cannot be split)
    J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, IA, C16, D0 = (
        "%%%d" % k for k in range(21))
    nkr = nkr_of(nk, jctr)
    KB = ["%%%d" % (21 + k) for k in range(nkr)]
    if prefetch:
        return ksa_prefetch(nk, J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, KB)
    out = []
    e = out.append
    # identity: dword w of lane l at area + 256 w + 4 l
    if b128:
        identity_b128(e, IA, C16, D0)
    else:
        identity(e, M, M0S, SB, ["%%%d" % (21 + nkr + k) for k in range(idregs)], m0_wait)
    # jctr: byte 3 of j counts positions (the key registers carry +3 / -1 in byte 3 for even / odd steps), so after
    # step 0 of group q it is i1 and after step 1 it is i0: both compares read it from j itself.  Bytes 1-2 absorb the
    # carries and W's byte 1 (at most 128 x 0x101 per KSA < 2^16: nothing reaches byte 3).
    e("v_mov_b32 %s, %s" % (J, "0xfe000000" if jctr else "0"))
    e("v_mov_b32 %s, 0x100" % W)         # group 0 = S[0] | S[1] << 8 of the identity
    IC = WN                              # vconst: (i0, i1) of the group in bytes 0, 1 of a VGPR, from the first
    FIRST_IC = 32 if vconst else 0       # group whose i1 is past the inline constants (0..64)
    if jctr:
        vconst = False
    if vconst:
        i0f = 2 * FIRST_IC
        # ic4 (round 4 A/B): (i0, i1) of two consecutive groups in bytes 0-3, bumped once per two groups
        e("v_mov_b32 %s, 0x%x" % (IC, (i0f | ((i0f + 1) << 8) | ((i0f + 2) << 16) | ((i0f + 3) << 24)) if ic4
                                  else (i0f | ((i0f + 1) << 8))))
    # d16 (round 4 A/B): x0 / x1 land in the low / high half of ONE register (ds_read_u8_d16 / _d16_hi) and the
    # merge is one v_perm whose selector is chosen by hit0 before the wait: SEL = hit0 ? [V1.b0, x0] : [x0, x1]
    SEL = X1 if d16 else None                          # x1's register is free: both bytes land in X0
    SEL_NOHIT, SEL_HIT = 0x0c0c0604, 0x0c0c0400        # v_perm(X, V1, sel): 4-7 = X bytes, 0-3 = V1 bytes
    SELHIT = "%%%d" % (21 + nkr)                       # input VGPRs holding SEL_HIT, SEL_NOHIT (rc4_dev.h,
    SELNO = "%%%d" % (22 + nkr)                        # RC4_KSA_SELHIT: VCC + a literal break the constant bus)

    def merge(q):
        """the deferred S[i0], S[i1] of group q as one u16 (VCC = hit0 of group q)"""
        if d16:
            e("v_perm_b32 %s, %s, %s, %s" % (M, X0, V1, SEL))
        else:
            e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))
            e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD "
              "src1_sel:DWORD" % (M, X1, X0))
        e("ds_write_b16 %s, %s offset:%d" % (LB, M, pos(2 * q)))

    def icsel(k):
        """SDWA byte of IC holding position i_k (k = 0, 1) of group q"""
        return "BYTE_%d" % (k + (2 if (ic4 and (q - FIRST_IC) % 2) else 0))
    RD0 = "ds_read_u8_d16" if d16 else "ds_read_u8"
    RD1 = "ds_read_u8_d16_hi" if d16 else "ds_read_u8"
    X1r = X0 if d16 else X1

    for q in range(128):
        i0, i1 = 2 * q, 2 * q + 1
        if q > 0:
            e("s_waitcnt lgkmcnt(%d)" % (0 if late_merge else 1))
        # split (round 4 A/B): j + K is formed off the chain (into the address register that is free by then), so the
        # chain pays one full-rate v_add after W / v1 arrives instead of a half-rate v_add3 -- same issue slots
        if split and q > 0:
            e("v_add_u32 %s, %s, %s" % (J, A1, W))
        else:
            e("v_add3_u32 %s, %s, %s, %s" % (J, J, W, KB[i0 % nkr]))
        if not vconst and not jctr:
            e("s_movk_i32 %s, %d" % (ST, i1))
        e(addr_lo(A0, J, LB, b3addr))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        if late_merge and q > 0:
            merge(q - 1)    # its S[i] stores precede this group's S[j] read (LDS in order), VCC still hit0(q-1)
        if early_read:      # the S[j] read one instruction earlier; the SALU move keeps the VCC distance
            e("ds_read_u8 %s, %s" % (X0, A0))
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (J, ST))
            e("ds_write_b8 %s, %s" % (A0, W))
            e("s_movk_i32 %s, %d" % (ST, i0))
        elif jctr:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:BYTE_3" % (J, J))
            e("ds_read_u8 %s, %s" % (X0, A0))
            e("ds_write_b8 %s, %s" % (A0, W))
        elif vconst:
            if q < FIRST_IC:
                e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i1))
            else:
                e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, icsel(1)))
            e("%s %s, %s" % (RD0, X0, A0))
            e("ds_write_b8 %s, %s" % (A0, W))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (J, ST))
            e("ds_read_u8 %s, %s" % (X0, A0))
            e("ds_write_b8 %s, %s" % (A0, W))
        if split:           # M is free between merges (its last reader, the previous u16 store, is long issued)
            e("v_add_u32 %s, %s, %s" % (M, J, KB[i1 % nkr]))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_0"
          % (V1, W, W))
        if split:
            e("v_add_u32 %s, %s, %s" % (J, M, V1))
        else:
            e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nkr]))
        if not early_read and not vconst and not jctr:
            e("s_movk_i32 %s, %d" % (ST, i0))
        e(addr_lo(A1, J, LB, b3addr))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        if early_read:
            e("ds_read_u8 %s, %s" % (X1, A1))
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (J, ST))
        elif jctr:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:BYTE_3" % (J, J))
            e("ds_read_u8 %s, %s" % (X1, A1))
        elif vconst:
            if q < FIRST_IC:
                e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i0))
            else:
                e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, icsel(0)))
            e("%s %s, %s" % (RD1, X1r, A1))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (J, ST))
            e("ds_read_u8 %s, %s" % (X1, A1))
        e("ds_write_b8 %s, %s" % (A1, V1))
        if d16:             # two LDS instructions after the hit0 compare: the VCC read is hazard-free
            e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (SEL, SELNO, SELHIT))
        if vconst and FIRST_IC <= q < 127:
            if not ic4:
                e("v_add_u32 %s, 0x202, %s" % (IC, IC))
            elif (q - FIRST_IC) % 2:
                e("v_add_u32 %s, 0x4040404, %s" % (IC, IC))
        if late_merge:
            if q < 127:
                e("ds_read_u16 %s, %s offset:%d" % (W, LB, pos(i0 + 2)))
            else:
                e("s_waitcnt lgkmcnt(0)")
                merge(q)
            continue
        if q < 127:
            e("ds_read_u16 %s, %s offset:%d" % (W, LB, pos(i0 + 2)))
            e("s_waitcnt lgkmcnt(1)")
        else:
            e("s_waitcnt lgkmcnt(0)")
        merge(q)
        if split and q < 127:   # the next group's j + K, off the chain (A1's last reader is several issues back)
            e("v_add_u32 %s, %s, %s" % (A1, J, KB[(i0 + 2) % nkr]))
    e("s_waitcnt lgkmcnt(0)")
    return out


def addr_lo(A, J, LB, b3addr):
    """A = (j & 3) | lanebase.  b3addr (round 4): as v_bitop3_b32 (LUT 0xea = (s0 & s1) | s2), which issues at full rate
    on gfx950 unless its three sources share a VGPR bank (profiles/vgpr_bank_r04.txt), where v_and_or_b32 is half rate"""
    if b3addr:
        return "v_bitop3_b32 %s, %s, 3, %s bitop3:0xea" % (A, J, LB)
    return "v_and_or_b32 %s, %s, 3, %s" % (A, J, LB)


def ksa_early_v1(nk):
    """vconst schedule with step 1's dependencies hoisted above step 0's LDS pair: the hit1 compare right after the
    j add, then the S[j0] address, v1 and the step-1 j add, and only then x0 = S[j0] / S[j0] = W.b0 -- the chain
    j0 -> v1 -> j1 -> S[j1] address no longer waits behind two LDS instructions (same instruction count)."""
    J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, IA, C16, D0 = (
        "%%%d" % k for k in range(21))
    KB = ["%%%d" % (21 + k) for k in range(nk)]
    out = []
    e = out.append
    identity(e, M, M0S, SB)
    e("v_mov_b32 %s, 0" % J)
    e("v_mov_b32 %s, 0x100" % W)
    IC = WN
    FIRST_IC = 32
    e("v_mov_b32 %s, 0x%x" % (IC, (2 * FIRST_IC) | ((2 * FIRST_IC + 1) << 8)))

    def cmp(i, sel):
        if q < FIRST_IC:
            e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, sel))

    for q in range(128):
        i0, i1 = 2 * q, 2 * q + 1
        if q > 0:
            e("s_waitcnt lgkmcnt(1)")
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, W, KB[i0 % nk]))
        cmp(i1, "BYTE_1")
        e("v_and_or_b32 %s, %s, 3, %s" % (A0, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_0"
          % (V1, W, W))
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nk]))
        e("ds_read_u8 %s, %s" % (X0, A0))
        e("ds_write_b8 %s, %s" % (A0, W))
        e("v_and_or_b32 %s, %s, 3, %s" % (A1, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        cmp(i0, "BYTE_0")
        e("ds_read_u8 %s, %s" % (X1, A1))
        e("ds_write_b8 %s, %s" % (A1, V1))
        if FIRST_IC <= q < 127:
            e("v_add_u32 %s, 0x202, %s" % (IC, IC))
        if q < 127:
            e("ds_read_u16 %s, %s offset:%d" % (W, LB, pos(i0 + 2)))
            e("s_waitcnt lgkmcnt(1)")
        else:
            e("s_waitcnt lgkmcnt(0)")
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
          % (M, X1, X0))
        e("ds_write_b16 %s, %s offset:%d" % (LB, M, pos(2 * q)))
    e("s_waitcnt lgkmcnt(0)")
    return out


def ksa_mskor(nk):
    """Round 5 A/B (VERDICT r4 "next" #2): each S[j] read + S[j] byte store fused into ONE ds_mskor_rtn_b32 on the
    dword holding S[j] -- MEM = (MEM & ~mask) | data, the old dword returned -- with mask = 0xff << 8 (j & 3) (v_bfm)
    and data = S[i] << 8 (j & 3); S[j] is the returned dword >> 8 (j & 3).  4 LDS operations per group instead of 6,
    for 6 more VALU (12 -> 18 per group): the S[j] address loses its (j & 3) byte-0 term (the address registers keep
    lanebase in bytes 0, 2, 3 across steps, only byte 1 is re-inserted), the shift amount sh = j << 3 (only its low
    5 bits are read), the mask, the data shift and one extract per step.  vconst compare constants as the default."""
    J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, IA, C16, D0 = (
        "%%%d" % k for k in range(21))
    # scratch VGPRs of this variant: the prefetch variant's SGPR-pair outputs are not used here, so the shift amounts,
    # masks and data words take the clobbered v60-v63 (sh0 / sh1 live until the extracts) and M / IA-free outputs
    SH0, SH1, MK, DT = "v60", "v61", "v62", "v63"
    KB = ["%%%d" % (21 + k) for k in range(nk)]
    out = []
    e = out.append
    identity(e, M, M0S, SB)
    e("v_mov_b32 %s, 0" % J)
    e("v_mov_b32 %s, 0x100" % W)
    e("v_mov_b32 %s, %s" % (A0, LB))      # byte 1 is replaced per step; bytes 0, 2, 3 stay lanebase's
    e("v_mov_b32 %s, %s" % (A1, LB))
    IC = WN
    FIRST_IC = 32
    e("v_mov_b32 %s, 0x%x" % (IC, (2 * FIRST_IC) | ((2 * FIRST_IC + 1) << 8)))

    def cmp(i, sel):
        if q < FIRST_IC:
            e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, sel))

    for q in range(128):
        i0, i1 = 2 * q, 2 * q + 1
        if q > 0:
            e("s_waitcnt lgkmcnt(1)")
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, W, KB[i0 % nk]))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        e("v_lshlrev_b32 %s, 3, %s" % (SH0, J))
        cmp(i1, "BYTE_1")
        e("v_bfm_b32 %s, 8, %s" % (MK, SH0))
        e("v_lshlrev_b32_sdwa %s, %s, %s dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
          % (DT, SH0, W))
        e("ds_mskor_rtn_b32 %s, %s, %s, %s" % (X0, A0, MK, DT))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_0"
          % (V1, W, W))
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nk]))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        e("v_lshlrev_b32 %s, 3, %s" % (SH1, J))
        cmp(i0, "BYTE_0")
        e("v_bfm_b32 %s, 8, %s" % (MK, SH1))
        e("v_lshlrev_b32 %s, %s, %s" % (DT, SH1, V1))
        e("ds_mskor_rtn_b32 %s, %s, %s, %s" % (X1, A1, MK, DT))
        if FIRST_IC <= q < 127:
            e("v_add_u32 %s, 0x202, %s" % (IC, IC))
        if q < 127:
            e("ds_read_u16 %s, %s offset:%d" % (W, LB, pos(i0 + 2)))
            e("s_waitcnt lgkmcnt(1)")
        else:
            e("s_waitcnt lgkmcnt(0)")
        e("v_lshrrev_b32 %s, %s, %s" % (X0, SH0, X0))
        e("v_lshrrev_b32 %s, %s, %s" % (X1, SH1, X1))
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
          % (M, X1, X0))
        e("ds_write_b16 %s, %s offset:%d" % (LB, M, pos(2 * q)))
    e("s_waitcnt lgkmcnt(0)")
    return out


def ksa_bytes(nk, idregs=0):
    """Round 5 A/B (--bytes): the S[i] pair of a group as two BYTE registers (two ds_read_u8 instead of one u16 read) and
    stored back as two bytes, so the select of v1 and the two merge selects are full-rate `v_cndmask_b32_e32` instead of
    half-rate SDWA forms: 6 half-rate + 6 full-rate VALU per group (36 VALU cycles) instead of 8 + 4 (40), for 8 LDS
    operations instead of 6.  Why: under load a chain's extra latency is issue contention (tools/rc4_probe_pmc.py: 22 %
    of wave-cycles ready-not-issued at 9 waves per CU), which the SIMD time of the half-rate ops drives."""
    J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, IA, C16, D0 = (
        "%%%d" % k for k in range(21))
    KB = ["%%%d" % (21 + k) for k in range(nk)]
    W0, W1, M1 = W, WN, "v60"          # W1 in the IC-free register of the vconst schedule's WN; M1 a clobbered VGPR
    IC = "v61"                         # the compare constants (i0, i1) in bytes 0, 1 (clobbered VGPR)
    out = []
    e = out.append
    identity(e, M, M0S, SB, ["%%%d" % (21 + nk + k) for k in range(idregs)])
    e("v_mov_b32 %s, 0" % J)
    e("v_mov_b32 %s, 0" % W0)          # S[0], S[1] of the identity
    e("v_mov_b32 %s, 1" % W1)
    FIRST_IC = 32
    e("v_mov_b32 %s, 0x%x" % (IC, (2 * FIRST_IC) | ((2 * FIRST_IC + 1) << 8)))

    def cmp(i, sel):
        if q < FIRST_IC:
            e("v_cmp_eq_u32_sdwa vcc, %s, %d src0_sel:BYTE_0 src1_sel:DWORD" % (J, i))
        else:
            e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:%s" % (J, IC, sel))

    for q in range(128):
        i0, i1 = 2 * q, 2 * q + 1
        if q > 0:
            e("s_waitcnt lgkmcnt(2)")          # W0, W1 landed; the previous group's two S[i] stores may be in flight
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, W0, KB[i0 % nk]))
        e(addr_lo(A0, J, LB, True))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        cmp(i1, "BYTE_1")
        e("ds_read_u8 %s, %s" % (X0, A0))
        e("ds_write_b8 %s, %s" % (A0, W0))
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (V1, W1, W0))        # v1 = hit1 ? S[i0] : S[i1]
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nk]))
        e(addr_lo(A1, J, LB, True))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        cmp(i0, "BYTE_0")
        e("ds_read_u8 %s, %s" % (X1, A1))
        e("ds_write_b8 %s, %s" % (A1, V1))
        if FIRST_IC <= q < 127:
            e("v_add_u32 %s, 0x202, %s" % (IC, IC))
        if q < 127:
            e("ds_read_u8 %s, %s offset:%d" % (W0, LB, pos(i0 + 2)))
            e("ds_read_u8 %s, %s offset:%d" % (W1, LB, pos(i0 + 3)))
            e("s_waitcnt lgkmcnt(2)")          # x0, x1 landed (the next pair may still be in flight)
        else:
            e("s_waitcnt lgkmcnt(0)")
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))         # S[i0] = hit0 ? v1 : x0
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M1, X1, X0))        # S[i1] = hit0 ? x0 : x1
        e("ds_write_b8 %s, %s offset:%d" % (LB, M, pos(i0)))
        e("ds_write_b8 %s, %s offset:%d" % (LB, M1, pos(i1)))
    e("s_waitcnt lgkmcnt(0)")
    return out


def identity(e, M, M0S, SB, ids=(), m0_wait=True):
    """ids (round 4 A/B, --idregs N): input VGPRs holding rows 0..N-1 of the identity (loop-invariant constants the
    kernel keeps in registers), so only the rows after them need the add chain"""
    e("s_mov_b32 %s, m0" % M0S)
    e("s_mov_b32 m0, %s" % SB)
    n = len(ids)
    # the v_mov is also the wait state an M0 write needs before an LDS instruction that reads M0 (ds_write_addtid): the
    # first round-4 --idregs build stored row 0 right behind the s_mov and lost it on the hardware (the write used the
    # old M0).  --no-m0-wait regenerates that schedule (round 5: tools/rc4_ksa_probe.hip shows rows 0 wrong on the
    # MI355X; tests/test_rc4_asm.py's hazard model rejects it)
    mov = "v_mov_b32 %s, 0x%x" % (M, (0x03020100 + 0x04040404 * n) & 0xffffffff)
    if m0_wait or not n:
        e(mov)
    for w in range(n):
        e("ds_write_addtid_b32 %s offset:%d" % (ids[w], 256 * w))
    if not (m0_wait or not n):
        e(mov)
    for w in range(n, 64):
        e("ds_write_addtid_b32 %s offset:%d" % (M, 256 * w))
        if w < 63:
            e("v_add_u32 %s, 0x4040404, %s" % (M, M))
    e("s_mov_b32 m0, %s" % M0S)


IDQ = ("v[60:63]", "v[60:61]", "v[62:63]", ("v60", "v61", "v62", "v63"))


def identity_b128(e, IA, C16, D0):
    """The identity as 16 ds_write_b128 instead of 64 ds_write_addtid_b32 + 63 v_add: lane l writes 16 bytes of row
    4t + l/16 (lanes 4(l%16) .. 4(l%16)+3 of it, which all hold the same identity dword) at IA = area + 256 (l/16)
    + 16 (l%16) + 1024 t; its data quad starts at 0x03020100 + 0x04040404 (l/16) (D0) in every dword and moves four
    rows on (+0x10101010 per dword) with two 64-bit adds.  LDS cycles: 16 x ~13 instead of 64 x 2 (the LDS pipe has
    room, LdsUtil 0.5); instructions: 50 instead of 131 per KSA."""
    quad, lo, hi, regs = IDQ
    for r in regs:
        e("v_mov_b32 %s, %s" % (r, D0))
    for t in range(16):
        e("ds_write_b128 %s, %s offset:%d" % (IA, quad, 1024 * t))
        if t < 15:
            e("v_lshl_add_u64 %s, %s, 0, %s" % (lo, lo, C16))
            e("v_lshl_add_u64 %s, %s, 0, %s" % (hi, hi, C16))


def ksa_prefetch(nk, J, W, X0, X1, V1, A0, A1, M, ST, M0S, WN, C0, C1, C2, C3, H0, LB, SB, KB):
    """The next group's pair is read at the START of a group -- its LDS latency overlaps the group instead of
    sitting on the j chain between groups -- and repaired afterwards for this group's two S[j] stores (j0 stored
    W.byte0, j1 stored v1; a later store wins).  W and Wn swap roles every group (no copy)."""
    out = []
    e = out.append
    identity(e, M, M0S, SB)
    e("v_mov_b32 %s, 0" % J)
    e("v_mov_b32 %s, 0x100" % W)
    regs = [W, WN]
    for q in range(128):
        i0, i1, p2, p3 = 2 * q, 2 * q + 1, 2 * q + 2, 2 * q + 3
        w, wn = regs[q & 1], regs[(q + 1) & 1]
        last = q == 127
        if not last:
            e("ds_read_u16 %s, %s offset:%d" % (wn, LB, pos(p2)))
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, w, KB[i0 % nk]))
        e("s_movk_i32 %s, %d" % (ST, i1))
        e("v_and_or_b32 %s, %s, 3, %s" % (A0, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A0, J))
        e("v_cmp_eq_u32_sdwa vcc, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (J, ST))
        e("ds_read_u8 %s, %s" % (X0, A0))
        e("ds_write_b8 %s, %s" % (A0, w))
        if not last:
            e("s_movk_i32 %s, %d" % (ST, p2))
            e("v_cmp_eq_u32_sdwa %s, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (C0, J, ST))
            e("s_movk_i32 %s, %d" % (ST, p3))
            e("v_cmp_eq_u32_sdwa %s, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (C1, J, ST))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:BYTE_0"
          % (V1, w, w))
        e("v_add3_u32 %s, %s, %s, %s" % (J, J, V1, KB[i1 % nk]))
        e("s_movk_i32 %s, %d" % (ST, i0))
        e("v_and_or_b32 %s, %s, 3, %s" % (A1, J, LB))
        e("v_lshrrev_b32_sdwa %s, 2, %s dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:BYTE_0"
          % (A1, J))
        e("v_cmp_eq_u32_sdwa %s, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (H0, J, ST))
        e("ds_read_u8 %s, %s" % (X1, A1))
        e("ds_write_b8 %s, %s" % (A1, V1))
        if not last:
            e("s_movk_i32 %s, %d" % (ST, p2))
            e("v_cmp_eq_u32_sdwa %s, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (C2, J, ST))
            e("s_movk_i32 %s, %d" % (ST, p3))
            e("v_cmp_eq_u32_sdwa %s, %s, %s src0_sel:BYTE_0 src1_sel:DWORD" % (C3, J, ST))
        # x0, x1 and the prefetched pair have landed (only the S[j1] store may still be in flight)
        e("s_waitcnt lgkmcnt(1)")
        e("s_mov_b64 vcc, %s" % H0)
        e("s_nop 1")
        e("v_cndmask_b32_e32 %s, %s, %s, vcc" % (M, X0, V1))
        e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD"
          % (M, X1, X0))
        e("ds_write_b16 %s, %s offset:%d" % (LB, M, pos(i0)))
        if not last:
            # S[p2] = byte 0 of wn, S[p3] = byte 1: j0's store (W.byte0) first, then j1's (v1)
            for cond, src, sel in ((C0, w, "BYTE_0"), (C2, V1, "BYTE_0")):
                e("s_mov_b64 vcc, %s" % cond)
                e("s_nop 1")
                e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_0 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 "
                  "src1_sel:%s" % (wn, wn, src, sel))
            for cond, src, sel in ((C1, w, "BYTE_0"), (C3, V1, "BYTE_0")):
                e("s_mov_b64 vcc, %s" % cond)
                e("s_nop 1")
                e("v_cndmask_b32_sdwa %s, %s, %s, vcc dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_1 "
                  "src1_sel:%s" % (wn, wn, src, sel))
    e("s_waitcnt lgkmcnt(0)")
    return out


def main():
    import sys
    early = "--early-read" in sys.argv      # A/B variants (tools/build_variant.sh with RC4_KSA_ASM_HEADER)
    late = "--late-merge" in sys.argv
    pre = "--prefetch" in sys.argv
    vconst = "--salu-consts" not in sys.argv
    b128 = "--b128-identity" in sys.argv
    ic4 = "--ic4" in sys.argv          # round 4 A/B: compare constants of two groups per register
    d16 = "--d16merge" in sys.argv     # round 4 A/B: d16 loads + one v_perm merge
    split = "--split-add" in sys.argv  # round 4 A/B: j + K off the chain, one full-rate v_add on it
    # the address's low byte by v_bitop3 (full rate) instead of v_and_or (half rate): default since round 4 (R3/R4 625.7
    # -> 628.3 M, R2 12.38 -> 12.39 G, profiles/ab_r24_b3addr_r04n.txt); --and-or restores the old form
    b3addr = "--and-or" not in sys.argv
    # identity rows 0..N-1 from N loop-invariant input VGPRs (rc4_dev.h idc[]): 23 fewer instructions per KSA.  Round 4
    # measured +0.4 % and saw the R4 verdict table fail on the MI355X; round 5 traced that failure to the schedule
    # without the M0 wait state (--no-m0-wait, tools/rc4_ksa_probe.hip: wrong S-boxes) and re-measured the fixed one:
    # green on the R2-R4 parity tests, R3/R4 625.5 vs 623.1 M, R2 12.34 vs 12.29 G (profiles/ab_r24_r05b.txt), so 24 is
    # the default since round 5 (--idregs 0: the add chain for every row, as before)
    own = any(f in sys.argv for f in ("--d16merge", "--b128-identity", "--prefetch", "--early-v1", "--mskor"))
    idregs = 0 if own else 24           # the variants with an identity / operand layout of their own take none
    if "--idregs" in sys.argv:
        idregs = int(sys.argv[sys.argv.index("--idregs") + 1])
        assert not (d16 and idregs), "--idregs puts its inputs where --d16merge puts its selectors"
    # --jctr: the j-counter schedule (measured round 3: 19 instructions per group but 1.3 % slower than the vconst
    # schedule on R3/R4 and R2 -- the compare reading j twice costs more than the v_add it saves); default: vconst
    jctr = "--jctr" in sys.argv and not (early or late or pre or b128 or "--salu-consts" in sys.argv)
    print("/* rc4_ksa_asm.h -- GENERATED by tools/gen_rc4_ksa_asm.py (see there for the schedule); do not edit. */")
    print("#ifndef DPRF_RC4_KSA_ASM_H")
    print("#define DPRF_RC4_KSA_ASM_H")
    print("/* key registers: 1 = byte 0 the key byte, bytes 1-2 zero, byte 3 the j-counter step (+3 even / -1 odd")
    print("   positions); 0 = the key byte in byte 0, anything above it.  RC4_KSA_NKR_5: registers of the 5-byte key */")
    print("#define RC4_KSA_KB_CTR %d" % (1 if jctr else 0))
    print("#define RC4_KSA_NKR_5 %d" % nkr_of(5, jctr))
    if idregs:
        print("#define RC4_KSA_IDREGS %d   /* identity rows 0..%d as input VGPRs after the keys (rc4_dev.h idc[]) */"
              % (idregs, idregs - 1))
        print("#define RC4_KSA_IDIN " + "".join(', "v"(idc[%d])' % k for k in range(idregs)))
    if d16:
        print("#define RC4_KSA_SELHIT 0x0c0c0400u   /* the block reads these two constants from the inputs after the keys */")
        print("#define RC4_KSA_SELNOHIT 0x0c0c0604u")
    for nk in KEYLENS:
        lines = (ksa_early_v1(nk) if "--early-v1" in sys.argv else ksa_mskor(nk) if "--mskor" in sys.argv else
                 ksa_bytes(nk, idregs) if "--bytes" in sys.argv else
                 ksa(nk, early, late, pre, vconst and not early, b128, jctr, ic4, d16, split, b3addr, idregs,
                     "--no-m0-wait" not in sys.argv))
        print("#define RC4_KSA_ASM_%d \\" % nk)
        for ln in lines:
            print('    "%s\\n\\t" \\' % ln)
        print('    ""')
    print("#endif")


if __name__ == "__main__":
    main()

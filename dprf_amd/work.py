"""Algorithmic work per candidate, for the VALU roofline (DESIGN.md section "Roofline").

Peak.  gfx950 issues one wave64 VALU instruction per SIMD every 2 cycles for FULL-RATE integer ops, i.e.
256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.64e12 lane-slots/s.  Measured on MI355X
(profiles/valu_issue_rates_r01.txt, tools/valu_peak.hip): v_add/v_sub/v_xor/v_and/v_or/v_not/v_lshrrev_b32
reach 96-98% of that; v_lshlrev_b32, v_alignbit (rotate), v_alignbyte, v_perm, v_bfe, v_add3, v_and_or,
v_lshl_or, v_sad_u8, v_mul_u32_u24 issue at half rate (2 slots).  v_bitop3_b32 issues at FULL rate (1 slot) whenever
its three sources are not all in one VGPR bank (register index mod 4): tools/valu_peak.hip mix "bitop3|xor indep"
76.1 T = 96.8 % (profiles/valu_mix_r04.txt), tools/vgpr_bank.hip 95-98 % with sources in banks 0,1,2 or 0,1,0 and
49 % only with 0,0,0 (profiles/vgpr_bank_r04.txt); the compiled KDF loops have no three-same-bank bitop3.  Until
round 5 this table charged it 1.7 slots -- the single-op probe's own register allocation (0,0,0), not the kernels'.

What the additive table does not model: a stream that MIXES half- and full-rate instructions issues slower than the
sum of their slots (profiles/valu_mix_r04.txt: 50/50 independent 3.74 cycles per wave-instruction against 3.0
additive; the ODF KDF loop's own 21-instruction pattern 3.75 against 3.24), so a kernel at the issue limit of its
own mix shows floor fractions ~0.85-0.9, not 1.0.

Floor.  The per-candidate work is the fewest issue slots the ALGORITHM needs on gfx950 with that cost
table, derived per primitive from its dataflow (sha1_floor() below does it exactly from which message
words are constant); a kernel that spends more slots than the floor shows a lower fraction of peak.

The survey's own per-unit figures (SURVEY.md 8(d), 2-input spec ops, 3-input op = 2) are SPEC, split (round 6,
VERDICT r5 #2) into the VALU ops the SIMDs issue (SPEC) and the LDS lane-operations of the table lookups (SPEC_LDS:
AES 160 / 224 per block, RC4 1,024 per KSA and 5 per PRGA byte), which the LDS executes, not the VALU: spec_frac
counts VALU ops only against the VALU peak, lds_spec_frac the LDS ops against one LDS per CU (32 lane-operations per
LDS-array cycle when conflict-free, MI355X_MICROARCH.md).

Instruction floor (round 6).  What bounds every VALU kernel here is its wave-instruction COUNT: the counters show
all of them issuing at ~3.9 cycles per wave-instruction (the mixed half/full-rate cadence of these streams,
profiles/valu_occ_r05t.txt), so the headroom is measured instructions per candidate against the fewest the algorithm
needs.  INSTR is that minimum per primitive in wave-instructions per lane, from the same dataflow functions as the
slot floor with unit "instr": every VALU instruction counts 1; three-input forms are used where gfx950 has them
(v_add3_u32 for a sum of three, v_bitop3_b32 for any 3-input bitwise function, v_lshl_add_u64 for a 64-bit add);
a rotate is one v_alignbit (a 64-bit rotate two); a table lookup's address one v_perm of the state byte and the
lane's table base (the split-table AES of the R6 and ODF kernels).  bench.py divides it by SQ_INSTS_VALU x 64 /
candidates of the profiled dispatch (instr_frac).
"""
import math

PEAK_SLOTS_PER_S = 256 * 4 * 32 * 2.4e9   # 78.64e12 full-rate VALU lane-slots/s
PEAK_LANE_INSTR_PER_S = PEAK_SLOTS_PER_S   # backwards-compatible name

# measured issue cost in full-rate slots
COST = {"add": 1.0, "xor": 1.0, "and": 1.0, "or": 1.0, "shr": 1.0, "shl": 2.0, "rot": 2.0, "bitop3": 1.0,
        "add3": 2.0, "perm": 2.0, "bfe": 2.0}


def _nadd(terms, unit):
    """a sum of `terms` values: terms - 1 additions, or (unit "instr") ceil((terms - 1) / 2) v_add3"""
    if terms <= 1:
        return 0
    return math.ceil((terms - 1) / 2) if unit == "instr" else (terms - 1) * COST["add"]


def sha1_floor(const_words, uniform_words=(), unit="slots"):
    """Issue-slot floor of one SHA-1 compression whose message words `const_words` are compile-time
    constants and `uniform_words` are wave-uniform (scalar unit, free for the VALU).  The chaining value
    is variable.  Per round: rol5 + f + (terms-1) additions + rol30; per schedule word: the XOR of its
    non-constant inputs + rol1.  unit "instr": wave-instructions instead (module docstring)."""
    ins_cost = {"slots": {1: 0, 2: COST["xor"], 3: COST["bitop3"], 4: COST["bitop3"] + COST["xor"]},
                "instr": {1: 0, 2: 1, 3: 1, 4: 2}}[unit]
    rot = COST["rot"] if unit == "slots" else 1
    f_ = COST["bitop3"] if unit == "slots" else 1
    kind = ["v"] * 16
    for i in const_words:
        kind[i] = "c"
    for i in uniform_words:
        kind[i] = "u"
    w = list(kind)
    slots = 0.0
    for t in range(80):
        if t >= 16:
            ins = [w[t - 3], w[t - 8], w[t - 14], w[t - 16]]
            nv = sum(1 for x in ins if x == "v")
            if nv == 0:
                wt = "u" if "u" in ins else "c"
            else:
                slots += ins_cost[nv] + rot
                wt = "v"
            w.append(wt)
        wt = w[t]
        # a' = rol5(a) + f(b,c,d) + e + K + W: K+W folds when W is not a VGPR value (rol5, f, e, [K+W] or K, W)
        terms = 4 if wt != "v" else 5
        slots += rot + f_ + _nadd(terms, unit) + rot
    return slots + 5 * (COST["add"] if unit == "slots" else 1)


def sha256_floor(unit="slots"):
    if unit == "instr":
        # Sigma1 (3 rotates + xor3) + Ch + t1 = h + S1 + Ch + K + W (2 add3) + Sigma0 + Maj + a' = t1 + S0 + Maj
        # (add3) + e' = d + t1; schedule: sigma0 / sigma1 (2 rotates + shift + xor3 each) + W (2 add3)
        return 64 * (4 + 1 + 2 + 4 + 1 + 1 + 1) + 48 * (4 + 4 + 2) + 8
    rnd = 3 * COST["rot"] + COST["bitop3"] + COST["bitop3"] + 4 * COST["add"] + 3 * COST["rot"] + COST["bitop3"] \
        + COST["bitop3"] + 2 * COST["add"] + COST["add"]
    sched = 2 * (2 * COST["rot"] + COST["shr"] + COST["bitop3"]) + 3 * COST["add"]
    return 64 * rnd + 48 * sched + 8 * COST["add"]


def sha256_dataflow(var_words, rounds=64, unit="floor"):
    """Work of one SHA-256 compression from the IV whose message words `var_words` vary per lane and whose other
    words are wave-uniform (held and combined in SGPRs by the scalar unit, free for the VALU), computing rounds
    0..rounds-1 and the schedule words they use.  Only operations with a per-lane input count.  unit "spec": the
    SURVEY 8(d) accounting (every 2-input op, rotate and shift 1: Sigma 5, Ch 4, Maj 5, sigma 5, 26 per round,
    13 per schedule word, 2,296 for the whole compression with its 8 final additions); unit "floor": issue slots
    with the COST table (Sigma = 3 rotates + bitop3, sigma = 2 rotates + shift + bitop3, Ch / Maj one bitop3).
    With rounds < 64 the final additions are the one compare word's (k_pdf_r5's early reject after round 60)."""
    if unit == "spec":
        big_s, ch, maj, small_s, add = 5, 4, 5, 5, 1
    elif unit == "instr":
        big_s, ch, maj, small_s, add = 4, 1, 1, 4, 1
    else:
        big_s = 3 * COST["rot"] + COST["bitop3"]
        ch = maj = COST["bitop3"]
        small_s = 2 * COST["rot"] + COST["shr"] + COST["bitop3"]
        add = COST["add"]

    def adds(n_var, n_other):
        if n_var == 0:
            return 0
        terms = n_var + (1 if n_other else 0)
        return math.ceil((terms - 1) / 2) if unit == "instr" else (terms - 1) * add

    w = [i in var_words for i in range(16)]
    work = 0.0
    for t in range(16, rounds):
        terms = [w[t - 2], w[t - 7], w[t - 15], w[t - 16]]
        work += (small_s if w[t - 2] else 0) + (small_s if w[t - 15] else 0) + adds(sum(terms), 4 - sum(terms))
        w.append(any(terms))
    a, b, c, d, e, f, g, h = [False] * 8          # the IV: constants
    for t in range(rounds):
        t1_var = [h, e, e or f or g, w[t]]        # h, Sigma1(e), Ch(e,f,g), W[t]  (+ K: a constant)
        work += (big_s if e else 0) + (ch if (e or f or g) else 0) + adds(sum(t1_var), 1)
        t1 = any(t1_var)
        t2 = a or b or c
        work += (big_s if a else 0) + (maj if t2 else 0)
        if unit == "instr":                        # a' = t1 + S0 + Maj in one v_add3 (or one add / none)
            work += 1 if (t1 or t2) else 0
        else:
            work += (add if a and t2 else 0) + (add if (t1 or t2) else 0)   # t2 = S0 + Maj, a' = t1 + t2
        work += add if (d or t1) else 0            # e' = d + t1
        h, g, f, e, d, c, b, a = g, f, e, (d or t1), c, b, a, (t1 or t2)
    return work + (8 if rounds == 64 else 1) * add


def sha512_floor(unit="slots"):
    if unit == "instr":
        # 64-bit values as register pairs: a rotate 2 v_alignbit, a shift 2, a 3-input bitwise op 2 v_bitop3, an add one
        # v_lshl_add_u64.  Round: S1 8 + Ch 2 + t1 (4 adds) + S0 8 + Maj 2 + a' (2 adds) + e' 1; schedule: s0, s1 8 each
        # + 3 adds
        return 80 * (8 + 2 + 4 + 8 + 2 + 2 + 1) + 64 * (8 + 8 + 3) + 8
    add64, rot64, shr64, x64 = 2 * COST["add"], 2 * COST["rot"], COST["rot"] + COST["shr"], 2 * COST["bitop3"]
    rnd = (3 * rot64 + x64) + x64 + 4 * add64 + (3 * rot64 + x64) + x64 + 2 * add64 + add64
    sched = 2 * (2 * rot64 + shr64 + x64) + 3 * add64
    return 80 * rnd + 64 * sched + 8 * add64


def md5_floor(n_const_words=0, unit="slots"):
    # F/G/H/I as one bitop3, a + f + (K + M) (K+M folds for constant M), rotate, + b
    if unit == "instr":   # a + f + K + M: 2 instructions (one v_add3 when K + M is one constant), rotate, + b
        return 64 * (1 + 2 + 1 + 1) - n_const_words * 4
    var = 64 * (COST["bitop3"] + 3 * COST["add"] + COST["rot"] + COST["add"])
    return var - n_const_words * 4 * COST["add"]


# AES with the four T-tables in LDS: 2 slots per table index (shift/and, or and + 16-bit shift),
# 2 x bitop3 per output column (4 table words + round key), last round S-box bytes reassembled.
AES_ROUND = 16 * 2 * COST["add"] + 4 * 2 * COST["bitop3"]
AES_LAST = 16 * 2 * COST["add"] + 4 * (3 * COST["perm"] + COST["xor"])
FLOOR = {
    "sha1c": sha1_floor(()),                                   # generic, all 16 words variable
    "sha1c_office_loop": sha1_floor(range(6, 16), (0,)),       # W0 = bswap(i) uniform, W1..W5 = H
    "sha1c_hmac20": sha1_floor(range(5, 16)),                  # PBKDF2 iteration: 20-byte message
    "sha256c": sha256_floor(), "sha512c": sha512_floor(), "md5c": md5_floor(), "md5c_16": md5_floor(12),
    "md5c_5": md5_floor(14),                                   # 5-byte message (R3 40-bit): words 2..15 constant
    "aes128_enc_block": 9 * AES_ROUND + AES_LAST + 4 * COST["xor"] + 4 * COST["xor"],   # + CBC xor
    "aes128_dec_block": 9 * AES_ROUND + AES_LAST + 4 * COST["xor"],
    "aes256_dec_block": 13 * AES_ROUND + AES_LAST + 8 * COST["xor"],                    # + CBC xor
    "aes128_keyexp": 10 * (4 * 2 * COST["add"] + 3 * COST["perm"] + 5 * COST["xor"]),
    "aes128_dec_sched": 9 * 4 * (4 * 2 * COST["add"] + 4 * 2 * COST["add"] + 2 * COST["bitop3"]),
    "aes256_keyexp_dec_sched": 7 * (8 * 2 * COST["add"] + 6 * COST["perm"] + 9 * COST["xor"])
    + 13 * 4 * (4 * 2 * COST["add"] + 4 * 2 * COST["add"] + 2 * COST["bitop3"]),
    # RC4: per KSA step j += S[i] + k (2 adds) and the S[j] address (and, shift, or = 4); the S[i]
    # address is an immediate.  PRGA byte: j update, two addresses, xor into the output byte.
    "rc4_ksa": 256 * (2 * COST["add"] + COST["and"] + COST["shl"] + COST["or"]) + 64 * COST["add"],
    "rc4_prga_byte": 2 * COST["add"] + 2 * (COST["and"] + COST["shl"] + COST["or"]) + COST["shl"] + COST["xor"],
}
# The instruction floor per primitive (module docstring).  AES with split T-tables in LDS: one v_perm address per
# lookup, two v_bitop3 (XOR3) per output column of a round; the last round's 16 S-box bytes assembled by 3 v_perm per
# word + the key XOR; the initial AddRoundKey 4 XOR; CBC 4 XOR.  Key schedules: 4 S-box addresses + 3 v_perm + 5 XOR
# per AES-128 round key (AES-256: 8 words per two round keys); the decryption schedule's InvMixColumns by 4 lookups
# + 2 XOR3 per word.  RC4: per KSA step j += S[i] + K (v_add3) and the S[j] address (2: the [i/4][lane][i%4] layout);
# the identity's 63 adds; per PRGA byte j += S[i], two addresses, the output lookup's address and the XOR.
AES_ROUND_I = 16 + 8
AES_LAST_I = 16 + 4 * (3 + 1)
INSTR = {
    "sha1c": sha1_floor((), unit="instr"),
    "sha1c_office_loop": sha1_floor(range(6, 16), (0,), unit="instr"),
    "sha1c_hmac20": sha1_floor(range(5, 16), unit="instr"),
    "sha256c": sha256_floor("instr"), "sha512c": sha512_floor("instr"), "md5c": md5_floor(0, "instr"),
    "md5c_16": md5_floor(12, "instr"), "md5c_5": md5_floor(14, "instr"),
    "aes128_enc_block": 9 * AES_ROUND_I + AES_LAST_I + 4 + 4,
    "aes128_dec_block": 9 * AES_ROUND_I + AES_LAST_I + 4,
    "aes256_dec_block": 13 * AES_ROUND_I + AES_LAST_I + 4 + 4,
    "aes128_keyexp": 10 * (4 + 3 + 5),
    "aes128_dec_sched": 9 * 4 * (4 + 2),
    "aes256_keyexp_dec_sched": 7 * (8 + 6 + 9) + 13 * 4 * (4 + 2),
    "rc4_ksa": 256 * (1 + 2) + 63,
    "rc4_prga_byte": 1 + 2 + 1 + 2 + 1,
}
# PDF R5 at its bench configuration (-pr 7: message words 0-1 carry the candidate, 2-15 are launch-uniform salt,
# padding and length; the compare of IV7 + e after round 60 rejects all but 2^-32 of the candidates): the dataflow
# floor of the early-reject compression (1,925 slots, against 2,200 for a compression of 16 per-lane words).
FLOOR["sha256c_r5"] = sha256_dataflow({0, 1}, rounds=61)
INSTR["sha256c_r5"] = sha256_dataflow({0, 1}, rounds=61, unit="instr")
# the floor a format's kernel is held to where its primitive runs on fewer per-lane inputs than the generic one
FLOOR_AS = {"pdf_r5": {"sha256c": "sha256c_r5"}}
SPEC = {   # SURVEY.md 8(d), VALU ops only (its AES / RC4 figures less their LDS ops, SPEC_LDS)
    "sha1c": 1001, "sha1c_office_loop": 1001, "sha1c_hmac20": 1001, "sha256c": 2296, "sha512c": 5840,
    "md5c": 532, "md5c_16": 532, "md5c_5": 532, "aes128_enc_block": 480, "aes128_dec_block": 480, "aes256_dec_block": 672,
    "aes128_keyexp": 0, "aes128_dec_sched": 0, "aes256_keyexp_dec_sched": 0, "rc4_ksa": 1280, "rc4_prga_byte": 11,
}
SPEC_LDS = {"aes128_enc_block": 160, "aes128_dec_block": 160, "aes256_dec_block": 224, "rc4_ksa": 1024,
            "rc4_prga_byte": 5}   # LDS lane-operations per unit
LDS_LANE_OPS_PER_CYCLE = 32       # one conflict-free LDS access of 32 lanes per LDS-array cycle (a wave64 op: 2)
# Formats whose spec count includes work the kernel by design does not execute (R5: rounds 61-63 after the early
# reject, and the launch-uniform message words on the scalar unit): their spec_frac is an EFFECTIVE rate, not a
# fraction of issued work.
SPEC_EFFECTIVE = {"pdf_r5"}

# Exact primitive counts per candidate (cross-checked against oracle.work_counts in
# tests/test_work_accounting.py).
COUNTS = {
    # Office, salt 16, L <= 19: H0 1 + 50,000 loop + final 1 + X1 2.  The verifier hash (1 more SHA1c)
    # is only reached by the 1/256 of candidates whose decrypted hash passes the zero-byte check (:168).
    "office": {"sha1c_office_loop": 50000, "sha1c": 4, "aes128_dec_block": 3, "aes128_keyexp": 1,
               "aes128_dec_sched": 1},
    # ODF standard stream (enc_len >= 1024): SHA256(pw) 1 + 1 KiB checksum 17;
    # PBKDF2: ipad/opad midstates 2 + 2 blocks x (U1: 2 + 1023 x 2)
    "odt": {"sha256c": 18, "sha1c": 4, "sha1c_hmac20": 4094, "aes256_dec_block": 64, "aes256_keyexp_dec_sched": 1},
    "odt_e": {"sha256c": 1, "sha1c": 4, "sha1c_hmac20": 4094, "aes256_dec_block": 1, "aes256_keyexp_dec_sched": 1},
    # PDF R3/R4: initial MD5 2 blocks + 50 (16-byte message); 20 x (KSA + 16 PRGA bytes).
    # MD5(PAD || ID) is document-constant (the reference recomputes it per candidate, :167); not counted.
    "pdf_r34": {"md5c": 2, "md5c_16": 50, "rc4_ksa": 20, "rc4_prga_byte": 320},
    # R3 with a 40-bit key (EVP_rc4_40, pdf...c:445-453): the 50 MD5s hash 5 bytes, the RC4 passes use 5-byte keys
    "pdf_r3_40": {"md5c": 2, "md5c_5": 50, "rc4_ksa": 20, "rc4_prga_byte": 320},
    "pdf_r2": {"md5c": 2, "rc4_ksa": 1, "rc4_prga_byte": 32},
    "pdf_r5": {"sha256c": 1},
    # PDF R6, L = 6: mean over 1,000 random lowercase candidates (69.9 rounds)
    "pdf_r6": {"sha256c": 1284.13, "sha512c": 1295.0, "aes128_enc_block": 15027.18, "aes128_keyexp": 69.89},
}
# The part of COUNTS done by the dominant kernel when a format runs as two kernels (Office/ODF: KDF kernel,
# then a short check kernel on the same stream); single-kernel formats are absent (all of COUNTS).
MAIN = {
    "office": {"sha1c_office_loop": 50000, "sha1c": 4},
    "odt": {"sha256c": 1, "sha1c": 4, "sha1c_hmac20": 4094},
    "odt_e": {"sha256c": 1, "sha1c": 4, "sha1c_hmac20": 4094},
}
# which resource bounds each format when no current rocprof profile says otherwise.  The RC4 formats saturate
# neither pipe (R3/R4 VALUBusy 0.73, LdsUtil 0.52: each wave's KSA is a chain of one dependent LDS round trip per
# two steps); VALU is the busier of the two, so that is what their fraction is quoted against.
BOUND = {"office": "valu", "odt": "valu", "odt_e": "valu", "pdf_r34": "valu", "pdf_r3_40": "valu", "pdf_r2": "valu",
         "pdf_r5": "valu", "pdf_r6": "valu"}


# LDS-array cycles per candidate of the RC4 formats, from MI355X_MICROARCH.md's LDS table: every byte / u16 / dword
# read or store of a wave takes 2 LDS-array cycles (two 32-lane groups, conflict-free: the [i/4][lane][i%4]
# layout), ds_write_addtid_b32 2.  This is what rocprof's LdsUtil (SQ_LDS_IDX_ACTIVE) counts: the model is
# within 1 % of it for R3/R4 and R2 (tests/test_work_accounting.py).  Until round 3 the model charged stores 4
# cycles -- that is a store's address + data transfer from the VGPRs (2 cycles per source dword, a path of its
# own with two halves per CU), not LDS-array time -- and overstated the LDS load by 46 % (0.76 vs LdsUtil 0.52).
#   R3/R4 per wave and KSA: identity 64 addtid + 256 S[j] reads + 256 S[j] stores + 128 u16 stores of the
#   group-deferred S[i] sides + 127 u16 group reads = 831 ops = 1,662 cycles; the early-reject PRGA-2 (swaps in
#   registers): one dword + 4 byte reads = 10; 20 passes; + the key hand-off per batch of 64 (4 dword stores by
#   the key wave, 4 dword reads by the RC4 wave) = 16.  Per wave, / 64 lanes.
#   R2: the same KSA + 4 PRGA bytes x (3 reads + 2 stores) x 2 + the hand-off 16.
LDS_CYCLES = {
    "pdf_r34": (20 * ((64 + 256 + 256 + 128 + 127) * 2 + 10) + 16) / 64.0,
    "pdf_r3_40": (20 * ((64 + 256 + 256 + 128 + 127) * 2 + 10) + 16) / 64.0,     # the same KSA schedule, 5-byte key
    "pdf_r2": ((64 + 256 + 256 + 128 + 127) * 2 + 4 * 5 * 2 + 16) / 64.0,
}
PEAK_LDS_CYCLES_PER_S = 256 * 2.4e9          # one LDS per CU

# The bound the RC4 formats can approach (round 5): neither pipe is full (VALUBusy 0.73, LdsUtil 0.52);
# each RC4 wave runs ONE dependent chain -- j -> S[j] address -> LDS read -> ... -> the next pair's LDS read -- and a CU
# holds 9 of them (a 16 KiB S-box per wave, ~152 KiB allocatable: tools/lds_occ.hip).  tools/rc4_ksa_probe.hip `time`
# runs the product's RC4 work per candidate (R3/R4: one pass = the asm KSA + the early-reject PRGA-2, 20 per candidate;
# R2: KSA + the 4-byte PRGA) with ONE wave per CU, so nothing queues in front of its LDS reads: the per-wave time is the
# chain's own latency.  9 chains per CU at that latency is the most this design delivers; the fraction below is how
# close the product comes (the rest is the 9 waves' mutual queueing on the LDS and the SIMDs).  Measured on MI355X,
# best of 3 launches of 4,000 passes after a 0.3 s warm-up (profiles/rc4_latency_r05.txt).
RC4_CHAINS_PER_CU = 9
RC4_PASSES = {"pdf_r34": 20, "pdf_r3_40": 20, "pdf_r2": 1}
RC4_PASS_NS_UNLOADED = {"pdf_r34": 8747.7, "pdf_r3_40": 8729.2, "pdf_r2": 8863.0}
RC4_LATENCY_SOURCE = "profiles/rc4_latency_r05.txt (the shipped --idregs 24 schedule, 1 wave/CU, mean of 2 launches)"


def lds_latency_bound(fmt, cus=256):
    """candidates/s per GPU if each CU ran RC4_CHAINS_PER_CU chains at the unloaded chain latency (None for formats
    without an RC4 chain)"""
    if fmt not in RC4_PASS_NS_UNLOADED:
        return None
    return cus * RC4_CHAINS_PER_CU * 64 / (RC4_PASSES[fmt] * RC4_PASS_NS_UNLOADED[fmt] * 1e-9)


def lds_frac(fmt, cand_per_s):
    """Fraction of the chip's LDS cycles the modelled LDS work of `cand_per_s` candidates takes (None for
    formats not bound by LDS)."""
    if fmt not in LDS_CYCLES:
        return None
    return cand_per_s * LDS_CYCLES[fmt] / PEAK_LDS_CYCLES_PER_S


def r5_floor(pwlen, unit="floor"):
    """PDF R5's early-reject compression for range candidates of `pwlen` bytes: the message words holding password
    bytes vary per lane (a word shared with the salt too), the rest are launch-uniform (the -pr 7 figure,
    words 0-1, is right for -pr 5..8 only)"""
    return sha256_dataflow(set(range(max(1, math.ceil(pwlen / 4)))), 61, "instr" if unit == "instr" else "floor")


def per_candidate(fmt, unit="floor", part="all", pwlen=None):
    """Per candidate: issue slots (unit "floor"), wave-instructions (unit "instr": the instruction floor), the survey's
    VALU spec ops (unit "spec") or its LDS lane-operations (unit "spec_lds"); part "main" counts only the dominant
    kernel's share (MAIN).  pwlen: the range length the floor of PDF R5 depends on (default: its bench's 7)."""
    table = {"floor": FLOOR, "instr": INSTR, "spec": SPEC, "spec_lds": SPEC_LDS}[unit]
    counts = MAIN.get(fmt, COUNTS[fmt]) if part == "main" else COUNTS[fmt]
    if fmt == "pdf_r5" and pwlen is not None and unit in ("floor", "instr"):
        return r5_floor(pwlen, unit) * counts["sha256c"]
    alias = FLOOR_AS.get(fmt, {}) if unit in ("floor", "instr") else {}
    return sum(table.get(alias.get(k, k), 0) * v for k, v in counts.items())


def lds_spec_frac(fmt, cand_per_s, part="all", cus=256, clock=2.4e9):
    """Fraction of the chip's LDS-array cycles (one LDS per CU) the survey's LDS lane-operations of `cand_per_s`
    candidates take (0 for formats without table lookups)."""
    return cand_per_s * per_candidate(fmt, "spec_lds", part) / LDS_LANE_OPS_PER_CYCLE / (cus * clock)

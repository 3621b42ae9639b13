"""Algorithmic work per candidate, for the VALU roofline (DESIGN.md section "Roofline").

Two units are kept side by side:

* SURVEY.md 8(d) "spec ops": 2-input 32-bit operation equivalents, a 3-input op counted as 2
  (SHA1c ~= 1001, SHA256c ~= 2296, ...).  This is the survey's per-unit figure.
* gfx950 "instruction floor": the fewest VALU lane-instructions the algorithm needs on gfx950, whose
  3-input instructions (v_bitop3_b32, v_add3_u32, v_alignbit_b32 as a rotate) retire several spec ops
  at once.  The roofline uses this unit, because the hardware peak (256 CU x 4 SIMD x 32 lanes x
  2.4 GHz = 78.64e12 lane-instructions/s) is an instruction-issue rate; a kernel executing more
  instructions than the floor shows up as a lower fraction, never a higher one.

Per-primitive floors (derivation in DESIGN.md):
  SHA1c   597  = 80 rounds x 5 (rol5, f, add3, add, rol30) + 64 schedule x 3 (xor3, xor, rol1) + 5
  SHA256c 1320 = 64 x 13 + 48 x 10 + 8
  SHA512c 3256 = 80 x 27 + 64 x 17 + 8          (64-bit ops on 32-bit lanes)
  MD5c    320  = 64 x 5
  AES-128 encrypt block 416, AES-128 decrypt block 412, AES-256 decrypt block 572 (T-tables in LDS:
  2 VALU per lookup + 2 xor3 per column, 40 per round)
  AES-128 key expansion 160; AES-256 expansion + decryption schedule 1300; AES-128 ditto 900
  RC4 KSA 832 VALU (+1088 LDS ops); RC4 PRGA byte 8 VALU (+5 LDS ops)
"""

PEAK_LANE_INSTR_PER_S = 256 * 4 * 32 * 2.4e9   # 78.64e12

FLOOR = {
    "sha1c": 597, "sha256c": 1320, "sha512c": 3256, "md5c": 320,
    "aes128_enc_block": 416, "aes128_dec_block": 412, "aes256_dec_block": 572,
    "aes128_keyexp": 160, "aes128_dec_sched": 900, "aes256_keyexp_dec_sched": 1300,
    "rc4_ksa": 832, "rc4_prga_byte": 8,
}
SPEC = {
    "sha1c": 1001, "sha256c": 2296, "sha512c": 5840, "md5c": 532,
    "aes128_enc_block": 640, "aes128_dec_block": 640, "aes256_dec_block": 896,
    "aes128_keyexp": 0, "aes128_dec_sched": 0, "aes256_keyexp_dec_sched": 0,
    "rc4_ksa": 2304, "rc4_prga_byte": 16,
}

# Exact primitive counts per candidate (cross-checked against oracle.work_counts in
# tests/test_work_accounting.py).  R6 depends on the candidate; its figure is the mean over 1,000
# random 6-letter candidates of the oracle's counts (tests/test_work_accounting.py regenerates it).
COUNTS = {
    # Office, salt 16, L <= 19: H0 1 + 50,000 + final 1 + X1 2; the verifier hash (1 more SHA1c) is
    # only reached by the 1/256 of candidates whose decrypted hash passes the zero-byte check (:168)
    "office": {"sha1c": 50004, "aes128_dec_block": 3, "aes128_keyexp": 1, "aes128_dec_sched": 1},
    # ODF standard stream (enc_len >= 1024): SHA256(pw) 1 + 1 KiB checksum 17; PBKDF2 2 + 2 x (2 + 1023 x 2)
    "odt": {"sha256c": 18, "sha1c": 4098, "aes256_dec_block": 64, "aes256_keyexp_dec_sched": 1},
    # ODF -e stream (enc_len 16)
    "odt_e": {"sha256c": 1, "sha1c": 4098, "aes256_dec_block": 1, "aes256_keyexp_dec_sched": 1},
    # PDF R3/R4: initial MD5 2 blocks + 50; 20 x (KSA + 16 PRGA bytes).  MD5(PAD || ID) is document-
    # constant (the reference recomputes it per candidate, :167); not counted.
    "pdf_r34": {"md5c": 52, "rc4_ksa": 20, "rc4_prga_byte": 320},
    "pdf_r2": {"md5c": 2, "rc4_ksa": 1, "rc4_prga_byte": 32},
    "pdf_r5": {"sha256c": 1},
    # PDF R6, L = 6: mean over 1,000 random lowercase candidates (69.9 rounds)
    "pdf_r6": {"sha256c": 1284.13, "sha512c": 1295.0, "aes128_enc_block": 15027.18, "aes128_keyexp": 69.89},
}


def per_candidate(fmt, unit="floor"):
    table = FLOOR if unit == "floor" else SPEC
    return sum(table[k] * v for k, v in COUNTS[fmt].items())

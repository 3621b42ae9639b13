#!/usr/bin/env python3
"""Where k_pdf_r6's VALU instructions go, per candidate (round 6, VERDICT r5 Weak #5 / Next #2).

rocprof counts 10.50 M wave-instructions per candidate lane for the R6 kernel (SQ_INSTS_VALU x 64 / candidates,
profiles/pmc_valu.json) against dprf_amd/work.py's instruction floor of 10.01 M.  This tool attributes the measured
count by primitive: it compiles probe kernels that run exactly one of the kernel's own primitives -- the same device
functions and asm blocks dprf_kernels_r6.hip uses (included verbatim), inputs loaded from memory so nothing folds --
counts the VALU instructions of each probe in the gfx950 disassembly (straight-line code: static = dynamic), subtracts
an empty probe's load/store overhead, and multiplies by the oracle-measured per-candidate counts of each primitive
(work.COUNTS["pdf_r6"], tests/test_work_accounting.py) plus the kernel's per-round extras (the family probe's key
expansion and first block, the period reads, K load/store).  What remains of the measured count is the slot
scheduler, the candidate starts and the loop control.

CPU only (hipcc cross-compiles gfx950).  Usage: tools/r6_instr_breakdown.py [measured_instr_per_candidate]
(default: profiles/pmc_valu.json's pdf_r6 figure).  Prints a JSON table; profiles/r6_instr_breakdown_r06.json keeps it.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
from dprf_amd import work  # noqa: E402

PROBES = r'''
#include "%(src)s"
#define IN(i) io[(i) * 64 + threadIdx.x]
#define OUT(i, v) io[(4096 + (i)) * 64 + threadIdx.x] = (v)
DEVI r6_lds probe_lds(const uint32_t *io) {
    r6_lds S; S.pat = IN(0); S.lanebase = IN(1); S.lanec = IN(2); S.base = IN(3); return S;
}
/* the empty probe: the same loads and stores, no work */
extern "C" __global__ void __launch_bounds__(768, 1) probe_empty(uint32_t *io) {
    for (int k = 0; k < 16; k++) OUT(k, IN(8 + k));
}
/* one AES-128 block of a round: CBC xor + the split-table cipher (R6_ENCRYPT), output to the SHA message */
extern "C" __global__ void __launch_bounds__(768, 1) probe_aes_block(uint32_t *io) {
    const r6_lds S = probe_lds(io);
    uint32_t rk[44], v[4], iv[4], y[4];
    for (int k = 0; k < 44; k++) rk[k] = IN(8 + k);
    for (int k = 0; k < 4; k++) { v[k] = IN(60 + k); iv[k] = IN(64 + k); }
    R6_ENCRYPT(S, rk, v, iv, y);
    for (int k = 0; k < 4; k++) OUT(k, y[k]);
}
/* one 16-byte block read from the slot's period column, range mode (r6_round UNI: 4 or 5 LDS words + 4 v_perm) */
extern "C" __global__ void __launch_bounds__(768, 1) probe_block_read(uint32_t *io, uint32_t o) {
    const r6_lds S = probe_lds(io);
    const uint32_t colbase = S.pat + S.lanebase;
    const uint32_t sel = 0x00010203u + (o & 3u) * 0x01010101u;
    const lds_u32 *col = L32(colbase + ((o >> 2) << 8));
    uint32_t lw[5], v[4];
    for (int k = 0; k < 4; k++) lw[k] = col[k * 64];
    lw[4] = (o & 3u) ? col[4 * 64] : lw[3];
    for (int k = 0; k < 4; k++) v[k] = perm(lw[k + 1], lw[k], sel);
    for (int k = 0; k < 4; k++) OUT(k, v[k]);
}
extern "C" __global__ void __launch_bounds__(768, 1) probe_sha256(uint32_t *io) {
    uint32_t hs[8], w[16];
    for (int k = 0; k < 8; k++) hs[k] = IN(8 + k);
    for (int k = 0; k < 16; k++) w[k] = IN(16 + k);
    sha256_compress(hs, w);
    for (int k = 0; k < 8; k++) OUT(k, hs[k]);
}
extern "C" __global__ void __launch_bounds__(768, 1) probe_sha512(uint32_t *io) {
    uint32_t hs[16], lo[16], hi[16];
    for (int k = 0; k < 16; k++) { hs[k] = IN(8 + k); lo[k] = IN(24 + k); hi[k] = IN(40 + k); }
    sha512_compress_pairs(hs, lo, hi);
    for (int k = 0; k < 16; k++) OUT(k, hs[k]);
}
extern "C" __global__ void __launch_bounds__(768, 1) probe_expand(uint32_t *io) {
    const r6_lds S = probe_lds(io);
    uint32_t key[4], rk[44];
    for (int k = 0; k < 4; k++) key[k] = IN(8 + k);
    R6_EXPAND(S, key, rk);
    for (int k = 0; k < 44; k++) OUT(k, rk[k]);
}
/* the per-round family probe (K load, key expansion, first block, byte sum mod 3) */
extern "C" __global__ void __launch_bounds__(768, 1) probe_family(uint32_t *io) {
    const r6_lds S = probe_lds(io);
    OUT(0, r6_family(S, IN(8)));
}
/* the per-round K store into the period column (r6_store_k) and K load (r6_load_k) */
extern "C" __global__ void __launch_bounds__(768, 1) probe_store_k(uint32_t *io, uint32_t bs) {
    const r6_lds S = probe_lds(io);
    uint32_t K[16];
    for (int k = 0; k < 16; k++) K[k] = IN(8 + k);
    r6_store_k(S, IN(30), bs, K, IN(31));
}
extern "C" __global__ void __launch_bounds__(768, 1) probe_load_k(uint32_t *io) {
    const r6_lds S = probe_lds(io);
    uint32_t K[8];
    r6_load_k(S, IN(8), K);
    for (int k = 0; k < 8; k++) OUT(k, K[k]);
}
'''


def valu_counts(asm):
    """VALU instructions per probe kernel in a gfx950 .s (function bodies between the symbol and .Lfunc_end)."""
    out, cur = {}, None
    for ln in asm.splitlines():
        m = re.match(r"^(probe_\w+):", ln)
        if m:
            cur = m.group(1)
            out[cur] = 0
            continue
        if cur and ln.startswith(".Lfunc_end"):
            cur = None
            continue
        t = ln.strip()
        if cur and t.startswith("v_"):
            out[cur] += 1
    return out


def compile_probes():
    src = os.path.join(HERE, "dprf_amd", "csrc", "dprf_kernels_r6.hip")
    with tempfile.TemporaryDirectory() as t:
        f = os.path.join(t, "probe.hip")
        open(f, "w").write(PROBES % {"src": src})
        s = os.path.join(t, "probe.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--offload-device-only",
                        "-S", "-I", os.path.join(HERE, "dprf_amd", "csrc"), f, "-o", s], check=True,
                       capture_output=True)
        return valu_counts(open(s).read())


def breakdown(measured=None):
    c = compile_probes()
    base = c["probe_empty"]
    net = {k: max(0, v - base) for k, v in c.items() if k != "probe_empty"}
    n = work.COUNTS["pdf_r6"]
    rounds = n["aes128_keyexp"]                        # one key expansion per round in the algorithm (the mean 69.9)
    rows = {
        "aes_block": {"per_unit": net["probe_aes_block"], "units": n["aes128_enc_block"]},
        "period_block_read": {"per_unit": net["probe_block_read"], "units": n["aes128_enc_block"]},
        "sha256c": {"per_unit": net["probe_sha256"], "units": n["sha256c"]},
        "sha512c": {"per_unit": net["probe_sha512"], "units": n["sha512c"]},
        "aes_key_expansion": {"per_unit": net["probe_expand"], "units": rounds},
        # r6_family per round: K load + key expansion + block + sum; r6_store_k per round; r6_load_k per round
        "family_probe": {"per_unit": net["probe_family"], "units": rounds},
        "k_store": {"per_unit": net["probe_store_k"], "units": rounds},
        "k_load": {"per_unit": net["probe_load_k"], "units": rounds},
    }
    floor = {"aes_block": work.INSTR["aes128_enc_block"], "sha256c": work.INSTR["sha256c"],
             "sha512c": work.INSTR["sha512c"], "aes_key_expansion": work.INSTR["aes128_keyexp"]}
    total = 0.0
    for k, r in rows.items():
        r["per_candidate"] = r["per_unit"] * r["units"]
        if k in floor:
            r["floor_per_unit"] = floor[k]
            r["floor_per_candidate"] = floor[k] * r["units"]
        total += r["per_candidate"]
    if measured is None:
        p = os.path.join(HERE, "profiles", "pmc_valu.json")
        measured = json.load(open(p)).get("pdf_r6", {}).get("valu_instr_per_candidate")
    out = {"probes_valu_instr": c, "empty_probe": base, "rows": rows, "attributed_per_candidate": total,
           "instr_floor_per_candidate": work.per_candidate("pdf_r6", "instr"),
           "measured_per_candidate": measured}
    if measured:
        out["unattributed_per_candidate"] = measured - total
        out["unattributed_frac"] = (measured - total) / measured
        out["shares_of_measured"] = {k: r["per_candidate"] / measured for k, r in rows.items()}
    return out


if __name__ == "__main__":
    m = float(sys.argv[1]) if len(sys.argv) > 1 else None
    print(json.dumps(breakdown(m), indent=1))

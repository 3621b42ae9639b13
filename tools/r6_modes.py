#!/usr/bin/env python3
"""PDF R6 kernel time per candidate, range mode (candidates enumerated inside k_pdf_r6<0>) vs list mode
(the same candidates packed on the host, k_pdf_r6<1>).  The two instantiations differ only in how a slot
gets its next password, and in register allocation (spills).  Usage on the box: tools/r6_modes.py"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    import bench
    from dprf_amd import _lib, brute_force
    S = bench.streams()
    fields = bench.quiet_fields(brute_force, S["pdf_synth_r6_ox"]["stream"])
    cs, n, start = bench.LOWER, 1 << 21, 1 << 22
    ctx = _lib.Context(fields, device=0)
    # list-mode blob of the same candidates (itertools.product order, pwlen 6)
    idx = np.arange(start, start + n, dtype=np.int64)
    chars = np.frombuffer(cs.encode(), dtype=np.uint8)
    words = np.empty((n, 6), dtype=np.uint8)
    v = idx.copy()
    for p in range(5, -1, -1):
        words[:, p] = chars[v % 26]
        v //= 26
    blob = words.tobytes()
    offs = np.arange(0, 6 * (n + 1), 6, dtype=np.uint64)
    out = {}
    for rep in range(2):
        hr, _, sr = ctx.search_range(cs, 6, start, n)
        hl, _, sl = ctx.verify_blob(blob, offs)
        assert [h - start for h in hr] == hl, (hr[:4], hl[:4])
        out["range_ms_%d" % rep] = sr["kernel_ms"]
        out["list_ms_%d" % rep] = sl["kernel_ms"]
    out["range_cand_per_s"] = n / (min(out["range_ms_0"], out["range_ms_1"]) / 1e3)
    out["list_cand_per_s"] = n / (min(out["list_ms_0"], out["list_ms_1"]) / 1e3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

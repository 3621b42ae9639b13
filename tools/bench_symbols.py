#!/usr/bin/env python3
"""Rates of range mode over a multi-byte charset (round 6): the device-spelled window (dprf_search_symbols, ABI 7)
against the same format's ASCII range mode (dprf_search_range) and the host-spelled list path it replaces
(payload.spell_utf8_parallel + dprf_verify_list), on bench.py's test documents.  One JSON line per format.

Usage (on the GPU box): python tools/bench_symbols.py [--formats odt,pdf_r5,...] [--seconds S]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402
from dprf_amd import _lib, brute_force  # noqa: E402
from dprf_amd.payload import spell_utf8_parallel  # noqa: E402

# 2-byte UTF-8 symbols, as many as the ASCII leg's charset where that fits
GREEK = "αβγδεζηθικλμνξοπρστυφχψω"
CYR = "абвгдежзийклмнопрстуфхцчшщъыьэюя"


def rate(fn, n):
    fn(n)                                           # warm-up (allocations, rate estimate)
    t = time.time()
    fn(n)
    return n / (time.time() - t)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--formats", default="odt,office,pdf_r34,pdf_r6,pdf_r2,pdf_r5")
    ap.add_argument("--seconds", type=float, default=2.0)
    a = ap.parse_args()
    S = bench.streams()
    for name in a.formats.split(","):
        stream_name, cs, pwlen, B, wkey, desc = bench.WORKLOADS[name]
        with contextlib.redirect_stdout(io.StringIO()):
            fields = brute_force.parse_verification_data(S[stream_name]["stream"])
        sym = (GREEK + CYR)[:len(cs)]
        with _lib.Context(fields, device=0) as ctx:
            n0 = 1 << 16
            t = time.time()
            ctx.search_range(cs, pwlen, 0, n0)
            r_est = n0 / max(1e-3, time.time() - t)
            n = int(max(1 << 16, min(B, r_est * a.seconds)))
            ascii_rate = rate(lambda k: ctx.search_range(cs, pwlen, 0, k), n)
            sym_rate = rate(lambda k: ctx.search_symbols(sym, pwlen, 0, k), n)
            hn = min(n, 1 << 22)

            def host(k):
                blob, offs = spell_utf8_parallel(sym, pwlen, 0, k, workers=min(16, os.cpu_count() or 1))
                ctx.verify_blob(blob, offs)
            host_rate = rate(host, hn)
        print(json.dumps({"format": name, "pwlen": pwlen, "symbols": len(sym), "bytes_per_symbol": 2,
                          "ascii_range": ascii_rate, "device_spelled": sym_rate, "host_spelled": host_rate,
                          "device_vs_ascii": sym_rate / ascii_rate, "device_vs_host": sym_rate / host_rate,
                          "candidates": n}), flush=True)


if __name__ == "__main__":
    main()

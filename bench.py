#!/usr/bin/env python3
"""bench.py -- verified candidates/s on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload odt|office|pdf_r34|pdf_r6|...]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (N=1 headline): BASELINE.json configs[1] -- ODF 1.2 AES-256 / PBKDF2-HMAC-SHA1 document,
`-pr 6` over the alnum charset (a-z A-Z 0-9, 62^6 = 56.8e9 candidates); the document is the reference's
own test file password.odt parsed the way server.py does (standard sha256-1k checksum stream).  A step
is one batch of B consecutive keyspace indices per GPU verified by libdprf.so's kernels; rank r takes
the r-th contiguous slice of each step's block (weak scaling: per-GPU work fixed).  After every step
the ranks all-reduce (RCCL, MIN) the lowest hit index -- the early-stop exchange of a real search.

Inputs are resident by construction: candidates are enumerated on the device from their index, so
nothing is copied host->device inside the timed region except the 320-byte kernel arguments.
"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

LOWER = "abcdefghijklmnopqrstuvwxyz"
ALNUM = LOWER + LOWER.upper() + "0123456789"
METRIC = "verified candidates/sec per format (Office/ODF/PDF) at 1/2/4/8 MI355X"

WORKLOADS = {
    # name: golden stream, charset, length, per-GPU batch per step, work-accounting key, description
    "odt": ("odt_testdoc_std", ALNUM, 6, 1 << 24, "odt",
            "configs[1]: ODF 1.2 AES-256-CBC / PBKDF2-HMAC-SHA1 (password.odt, sha256-1k stream), -pr 6 alnum"),
    "office": ("office_testdoc", LOWER, 4, 26 ** 4, "office",
               "configs[0]: ECMA-376 Standard Encryption (password.docx), -pr 4 lowercase"),
    "pdf_r34": ("pdf_testdoc_r4", ALNUM, 7, 1 << 28, "pdf_r34",
                "configs[2]: PDF 1.7 V4/R4 (password_1.7_v4_r4.pdf), MD5 x50 + RC4 x20, -pr 7 alnum"),
    "pdf_r6": ("pdf_synth_r6_ox", LOWER, 6, 1 << 22, "pdf_r6",
               "configs[3]: PDF 2.0 R6 hardened hash (synthetic document), -pr 6 lowercase"),
    "pdf_r2": ("pdf_testdoc_r2", ALNUM, 7, 1 << 30, "pdf_r2", "PDF 1.3 V1/R2 (password_1.3_v1_r2.pdf), -pr 7 alnum"),
    "pdf_r5": ("pdf_synth_r5_cat", ALNUM, 7, 1 << 31, "pdf_r5", "PDF R5 (synthetic document), -pr 7 alnum"),
    "odt_e": ("odt_testdoc_e", ALNUM, 6, 1 << 24, "odt_e", "ODF -e 2-byte stream (brute_force.py:239 path), -pr 6 alnum"),
}
# rocprofv3 name of the dominant kernel per libdprf kernel family (the one "roofline" times)
DOMINANT = {"office_std": "k_office_kdf", "odf_aes256": "k_odt_kdf", "pdf_r24": "k_pdf_r24", "pdf_r5": "k_pdf_r5",
            "pdf_r6": "k_pdf_r6"}
SIDE_FORMATS = ["office", "pdf_r34", "pdf_r6", "pdf_r2", "pdf_r5"]


def streams():
    return json.load(open(os.path.join(HERE, "tests", "golden", "streams.json")))


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    return int(os.environ.get("RANK", "0")), ws, int(os.environ.get("LOCAL_RANK", "0"))


def quiet_fields(brute_force, stream):
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        return brute_force.parse_verification_data(stream)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------ CPU baseline (reference verify())
def ref_callable(fmt_fields):
    """The reference's own verify() compiled from /root/reference (oracle/ref.mk -> oracle/_ref), called
    in-process with the argv strings brute_force.py builds (brute_force.py:163-197)."""
    f = fmt_fields
    ref = os.path.join(HERE, "oracle", "_ref")
    lib = {"office": "libref_office.so", "odt": "libref_odt.so", "pdf": "libref_pdf.so"}[f[0]]
    path = os.path.join(ref, lib)
    if not os.path.exists(path):
        return None
    L = ctypes.CDLL(path)
    if f[0] == "pdf":
        L.ref_load_legacy()
    v = L.verify
    v.restype = ctypes.c_int
    b = lambda s: str(s).encode()
    if f[0] == "office":
        args = [b(f[5]), int(f[4]), b(f[6]), len(f[6]) // 2, b(f[7]), len(f[7]) // 2, int(f[3]), int(f[2])]
        v.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                      ctypes.c_int, ctypes.c_int, ctypes.c_int]
    elif f[0] == "odt":
        args = [b(f[2]), b(f[3]), b(f[4]), b(f[5]), int(f[6])]
        v.argtypes = [ctypes.c_char_p] * 5 + [ctypes.c_int]
    else:
        args = [int(f[1]), int(f[2]), int(f[3]), int(f[4]), int(f[5]), int(f[6]), b(f[7]), int(f[8]), b(f[9]),
                int(f[10]), b(f[11])]
        v.argtypes = [ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                                               ctypes.c_int, ctypes.c_char_p]
    return lambda pw: v(pw, *args)


def _cpu_worker(job):
    """One baseline worker process: verify candidates t, t+P, t+2P, ... until the deadline."""
    fields, charset, pwlen, t, procs, deadline = job
    from dprf_amd.brute_force import _index_to_password
    fn = ref_callable(fields)
    if fn is None:
        sys.path.insert(0, os.path.join(HERE, "oracle"))
        import pyoracle
        ctx = pyoracle.Ctx(fields)
        fn = ctx.verify
    n, i = 0, t
    while time.time() < deadline:
        fn(_index_to_password(i, charset, pwlen).encode())
        n += 1
        i += procs
    return n


def _popen_worker(job):
    """One worker of the reference's process model: Popen + wait of the reference verifier executable per
    candidate (brute_force.py:123-140, argv of :163-197), candidates t, t+P, ... until the deadline."""
    fields, charset, pwlen, t, procs, deadline = job
    import subprocess
    from dprf_amd.brute_force import _index_to_password
    sys.path.insert(0, os.path.join(HERE, "tests", "golden"))
    from make_golden import ENV, ref_argv
    n, i = 0, t
    while time.time() < deadline:
        subprocess.run(ref_argv(fields, _index_to_password(i, charset, pwlen)), env=ENV,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        n += 1
        i += procs
    return n


def reference_process_model(fields, charset, pwlen, seconds=2.0, procs=4):
    """The reference engine's own cost structure: 4 worker processes (brute_force.py:70-73), one fork/exec
    of the compiled reference verifier per candidate.  Python 3 drives it (there is no Python 2.7 here)."""
    import multiprocessing as mp
    exe = os.path.join(HERE, "oracle", "_ref", {"office": "msoffcrypto", "odt": "odt", "pdf": "pdf"}[fields[0]])
    if not os.path.exists(exe):
        return None
    with mp.get_context("spawn").Pool(procs) as pool:
        t0 = time.time()
        counts = pool.map(_popen_worker, [(fields, charset, pwlen, t, procs, t0 + seconds) for t in range(procs)])
        dt = time.time() - t0
    n = sum(counts)
    return {"value": n / dt, "unit": "candidates/s", "cores": procs, "kind": "reference",
            "sample": "%d candidates in %.1f s: brute_force.py's 4 worker processes, one Popen of the reference "
                      "verifier executable (compiled from /root/reference) per candidate" % (n, dt)}


def cpu_baseline(fields, charset, pwlen, seconds=1.5, procs=None):
    """The reference's verify() on the host cores, one worker PROCESS per core (the reference's own process
    model, brute_force.py:70-73, minus its per-candidate fork/exec), for a bounded time over the first
    indices of the workload keyspace.  Run before anything touches the GPU (workers are spawned)."""
    import multiprocessing as mp
    kind = "reference" if ref_callable(fields) is not None else "port"
    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    procs = procs or max(1, min(16, ncpu))
    with mp.get_context("spawn").Pool(procs) as pool:
        pool.map(_cpu_worker, [(fields, charset, pwlen, t, procs, time.time() + 0.2) for t in range(procs)])  # warm
        t0 = time.time()
        counts = pool.map(_cpu_worker, [(fields, charset, pwlen, t, procs, t0 + seconds) for t in range(procs)])
        dt = time.time() - t0
    n = sum(counts)
    return {"value": n / dt, "unit": "candidates/s", "cores": procs, "kind": kind,
            "sample": "%d candidates (the first indices of the workload keyspace) in %.1f s on %d worker processes: "
                      "the reference's verify() %s in-process, no per-candidate fork/exec" % (
                          n, dt, procs, "compiled from /root/reference" if kind == "reference" else "(C port)")}


# ------------------------------------------------------------------ GPU timing
def shard(step, rank, world, batch, space):
    """Keyspace slice of `rank` at `step`: step s covers the contiguous block [s*world*B, (s+1)*world*B)
    (wrapped inside the keyspace) and rank r takes its r-th B-sized piece -- contiguous shards, no
    overlap, no gaps, and no data exchange between ranks."""
    start = ((step * world + rank) * batch) % max(1, space - batch)
    return start, min(batch, space - start)


def run_workload(name, ctx, rank, world, steps, warmup, sync, allreduce_min, batch=None):
    _, cs, pwlen, B, _, _ = WORKLOADS[name]
    B = batch or B
    space = len(cs) ** pwlen
    while space < world * B:     # e.g. Office -pr 4 (one batch) at N > 1: the next length keeps the shards disjoint
        pwlen += 1
        space = len(cs) ** pwlen
    stats = []
    lowest = None

    def step(s):
        start, n = shard(s, rank, world, B, space)
        hits, _, st = ctx.search_range(cs, pwlen, start, n)
        first = hits[0] if hits else (1 << 62)
        return allreduce_min(first), st

    for s in range(warmup):
        step(s)
    sync()
    t0 = time.perf_counter()
    for s in range(warmup, warmup + steps):
        low, st = step(s)
        stats.append(st)
        lowest = low if lowest is None else min(lowest, low)
    sync()
    dt = time.perf_counter() - t0
    return dt, stats, lowest, pwlen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="odt", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU candidates per step (default per workload)")
    ap.add_argument("--no-side", action="store_true", help="skip the per-format side measurements")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    args = ap.parse_args()

    rank, world, local = dist_env()
    import torch
    from dprf_amd import _lib, brute_force, work

    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)

    def sync():
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()

    def allreduce_min(v):
        if not dist:
            return v
        t = torch.tensor([v], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    def allreduce_max(v):
        if not dist:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    S = streams()
    stream_name, cs, pwlen, B, wkey, desc = WORKLOADS[args.workload]
    fields = quiet_fields(brute_force, S[stream_name]["stream"])

    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(fields, cs, pwlen, seconds=args.cpu_seconds)
        pm = reference_process_model(fields, cs, pwlen)
        if pm:
            cpu["reference_process_model"] = pm
        log("cpu baseline:", cpu)

    ctx = _lib.Context(fields, device=local)
    B = args.batch or B
    dt, stats, lowest, pwlen = run_workload(args.workload, ctx, rank, world, args.steps, args.warmup, sync, allreduce_min, B)
    dt_max = allreduce_max(dt)
    cands = sum(s["candidates"] for s in stats)
    total = cands * world
    launches = sum(s["launches"] for s in stats)
    kern_ms = sum(s["kernel_ms"] for s in stats)
    main_ms = sum(s["main_kernel_ms"] for s in stats)
    avg_launch_ms = main_ms / max(1, launches)          # dominant kernel alone (Office/ODF: the KDF kernel)
    per_launch = cands / max(1, launches)
    floor = work.per_candidate(wkey, part="main")
    achieved = per_launch * floor / (avg_launch_ms / 1e3)
    peak = work.PEAK_LANE_INSTR_PER_S
    traffic = None
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        traffic = json.load(open(pmc)).get(args.workload, {}).get("bytes_per_launch")

    side = {}
    if not args.no_side:
        for name in SIDE_FORMATS:
            if name == args.workload:
                continue
            sn, scs, spl, sB, skey, sdesc = WORKLOADS[name]
            sf = quiet_fields(brute_force, S[sn]["stream"])
            sctx = _lib.Context(sf, device=local)
            sdt, sst, _, spl = run_workload(name, sctx, rank, world, 2, 1, sync, allreduce_min)
            sdt = allreduce_max(sdt)
            sc = sum(s["candidates"] for s in sst)
            sl = sum(s["launches"] for s in sst)
            skm = sum(s["kernel_ms"] for s in sst)
            side[name] = {"value": sc * world / sdt, "unit": "candidates/s", "kernel": sctx.kernel, "config": sdesc,
                          "pwlen": spl,
                          "avg_launch_ms": skm / max(1, sl),
                          "valu_floor_frac": (sc / max(1, sl)) * work.per_candidate(skey) / (skm / max(1, sl) / 1e3) / peak}
            if work.BOUND.get(skey) == "lds":
                side[name]["lds_cycle_frac"] = work.lds_frac(skey, (sc / max(1, sl)) / (skm / max(1, sl) / 1e3))
            sctx.close()

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": total / dt_max,
            "unit": "candidates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic: consecutive keyspace indices enumerated on the device, verified against the "
                    "reference's test document",
            "config": {"workload": args.workload, "description": desc, "document": stream_name,
                       "charset": "alnum (a-z A-Z 0-9)" if cs == ALNUM else "lowercase", "pwlen": pwlen,
                       "batch_per_gpu": B, "kernel": ctx.kernel, "parallelism": "keyspace shards x%d" % world},
            "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": peak / 1e12,
                         "unit": "T VALU lane-instr/s (gfx950 instruction floor of the algorithm)",
                         "frac": achieved / peak, "traffic": traffic,
                         "kernel": DOMINANT.get(ctx.kernel, ctx.kernel),
                         "kernel_avg_ms": avg_launch_ms, "candidates_per_launch": per_launch,
                         "floor_instr_per_candidate": floor,
                         "all_kernels_avg_ms": kern_ms / max(1, launches),
                         "all_kernels_frac": cands * work.per_candidate(wkey) / (kern_ms / 1e3) / peak,
                         "spec_ops_per_candidate": work.per_candidate(wkey, "spec"),
                         "lds_cycle_frac": work.lds_frac(wkey, per_launch / (avg_launch_ms / 1e3))},
            "cpu_baseline": cpu,
            "per_format": side,
            "lowest_hit_index": None if lowest is None or lowest >= (1 << 62) else lowest,
        }
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

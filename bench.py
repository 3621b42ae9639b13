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
    "pdf_r6": ("pdf_synth_r6_ox", LOWER, 6, 1 << 25, "pdf_r6",   # 2^25: one ~9 s launch per step
               "configs[3]: PDF 2.0 R6 hardened hash (synthetic document), -pr 6 lowercase"),
    "pdf_r2": ("pdf_testdoc_r2", ALNUM, 7, 1 << 30, "pdf_r2", "PDF 1.3 V1/R2 (password_1.3_v1_r2.pdf), -pr 7 alnum"),
    "pdf_r5": ("pdf_synth_r5_cat", ALNUM, 7, 1 << 31, "pdf_r5", "PDF R5 (synthetic document), -pr 7 alnum"),
    "odt_e": ("odt_testdoc_e", ALNUM, 6, 1 << 24, "odt_e", "ODF -e 2-byte stream (brute_force.py:239 path), -pr 6 alnum"),
    # configs[2] names "PDF 1.4 R3/R4": the V2/R3 128-bit path (synthetic 1.4 document) and R3 with a 40-bit key
    # (EVP_rc4_40, pdf...c:445-453) beside the R4 test document (round 4)
    "pdf_r3": ("pdf_synth_r3_l128_abc", ALNUM, 7, 1 << 28, "pdf_r34",
               "configs[2]: PDF 1.4 V2/R3 128-bit key (synthetic document), -pr 7 alnum"),
    "pdf_r3_40": ("pdf_synth_r3_l40_cab", ALNUM, 7, 1 << 28, "pdf_r3_40",
                  "configs[2]: PDF 1.4 V2/R3 40-bit key (synthetic document), -pr 7 alnum"),
}
# rocprofv3 name of the dominant kernel per libdprf kernel family (the one "roofline" times)
DOMINANT = {"office_std": "k_office_kdf", "odf_aes256": "k_odt_kdf", "pdf_r24": "k_pdf_r24", "pdf_r5": "k_pdf_r5",
            "pdf_r6": "k_pdf_r6"}
SIDE_FORMATS = ["office", "odt_e", "pdf_r34", "pdf_r3", "pdf_r3_40", "pdf_r6", "pdf_r2", "pdf_r5"]
# keys of a rocprof record kept in the bench line (the whole record goes to the stderr detail line)
ROCPROF_KEYS = ("valu_busy", "valu_utilization", "lds_util", "wait_any_frac", "lds_bank_conflict_frac",
                "effective_clock_GHz", "source", "build", "stale")


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


def cpu_share():
    """(nproc, cores this job may use).  On the GPU box nproc is the whole machine while the job's share is
    16 CPUs (the pool's rule; exported there as OMP_NUM_THREADS), so the share is the cgroup CPU quota if
    one is set, else OMP_NUM_THREADS, else the affinity mask."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    share = aff
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            share = min(share, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        if os.environ.get("OMP_NUM_THREADS", "").isdigit():
            share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    else:
        if q == "max" and os.environ.get("OMP_NUM_THREADS", "").isdigit():
            share = min(share, int(os.environ["OMP_NUM_THREADS"]))
    return os.cpu_count() or aff, max(1, share)


def reference_process_model(fields, charset, pwlen, seconds=2.0, procs=4):
    """The reference engine's own cost structure: 4 worker processes (brute_force.py:70-73), one fork/exec
    of the compiled reference verifier per candidate (brute_force.py:123-140, 163-197).  Python 3 drives it
    (there is no Python 2.7 here)."""
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
    """The reference's verify() on `procs` worker PROCESSES (the reference's own process model,
    brute_force.py:70-73, minus its per-candidate fork/exec), for a bounded time over the first indices of
    the workload keyspace.  Run before anything touches the GPU (workers are spawned)."""
    import multiprocessing as mp
    kind = "reference" if ref_callable(fields) is not None else "port"
    procs = procs or cpu_share()[1]
    with mp.get_context("spawn").Pool(procs) as pool:
        pool.map(_cpu_worker, [(fields, charset, pwlen, t, procs, time.time() + 0.2) for t in range(procs)])  # warm
        t0 = time.time()
        counts = pool.map(_cpu_worker, [(fields, charset, pwlen, t, procs, t0 + seconds) for t in range(procs)])
        dt = time.time() - t0
    n = sum(counts)
    return {"value": n / dt, "unit": "candidates/s", "cores": procs, "kind": kind,
            "sample": "%d candidates (the first indices of the workload keyspace) in %.1f s on %d worker process%s: "
                      "the reference's verify() %s in-process, no per-candidate fork/exec" % (
                          n, dt, procs, "" if procs == 1 else "es",
                          "compiled from /root/reference" if kind == "reference" else "(C port)")}


def cpu_baselines(fields, charset, pwlen, seconds=1.5, process_model=True):
    """SURVEY.md 8(d) CPU path: the reference's verify() on 1 worker, on all cores of this job's share, and
    the reference's 4-process Popen-per-candidate model, with nproc and the share stated.  `value` is the
    all-cores figure."""
    nproc, share = cpu_share()
    allc = cpu_baseline(fields, charset, pwlen, seconds=seconds, procs=share)
    one = cpu_baseline(fields, charset, pwlen, seconds=seconds, procs=1)
    out = dict(allc)
    out.update({"nproc": nproc, "cpu_share": share, "all_cores": allc, "one_worker": one})
    if process_model:
        out["process_model_4"] = reference_process_model(fields, charset, pwlen, seconds=seconds)
    return out


# ------------------------------------------------------------------ GPU timing
def shard(step, rank, world, batch, space):
    """Keyspace slice of `rank` at `step`: step s covers the contiguous block [s*world*B, (s+1)*world*B)
    (wrapped inside the keyspace) and rank r takes its r-th B-sized piece -- contiguous shards, no
    overlap, no gaps, and no data exchange between ranks."""
    start = ((step * world + rank) * batch) % max(1, space - batch)
    return start, min(batch, space - start)


def run_workload(name, ctx, rank, world, steps, warmup, sync, allreduce_min, batch=None, ndev=1, stop_on_first=False):
    """W untimed + K timed steps of `name` on this rank.  A step verifies B consecutive indices per GPU
    (ndev GPUs in this process: one multi-device library call covers ndev * B) through
    brute_force.search_round -- the exact call the product's range mode makes per round -- then the ranks
    all-reduce (MIN) the lowest hit index, the early-stop exchange of a sharded search."""
    from dprf_amd import brute_force
    _, cs, pwlen, B, _, _ = WORKLOADS[name]
    B = (batch or B) * ndev
    space = len(cs) ** pwlen
    while space < world * B:     # e.g. Office -pr 4 (one batch) at N > 1: the next length keeps the shards disjoint
        pwlen += 1
        space = len(cs) ** pwlen
    stats = []
    lowest = None

    def step(s):
        start, n = shard(s, rank, world, B, space)
        idx, st = brute_force.search_round(ctx, cs, pwlen, start, n, stop_on_first=stop_on_first)
        return allreduce_min(idx if idx is not None else (1 << 62)), st

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


def launch_traffic(path, workload, per_launch, build):
    """HBM bytes (FETCH_SIZE + WRITE_SIZE) of the dominant kernel per launch of THIS run: the profile's bytes
    per candidate x this run's candidates per launch (the adaptive chunking may size launches differently
    from the profiled run).  Returns (bytes or None, record): the record names the profile and the build it
    measured, and carries "stale": true when that build is not the library this run timed."""
    if not os.path.exists(path):
        return None, None
    tr = json.load(open(path)).get(workload)
    if not tr:
        return None, None
    rec = dict(tr, stale=tr.get("build") != build)
    if tr.get("bytes_per_candidate") is not None and per_launch:
        return tr["bytes_per_candidate"] * per_launch, rec
    return tr.get("bytes_per_launch"), rec


def pmc_summary(workload, build):
    """rocprof-derived counters of the workload's dominant kernel (profiles/pmc_valu.json, written by
    tools/pmc_traffic.py from the tools/profile_gpu.sh passes): VALUBusy, VALUUtilization, LDS busy -- with the
    build fingerprint of the library they were measured on and "stale": true when it is not this run's."""
    p = os.path.join(HERE, "profiles", "pmc_valu.json")
    if not os.path.exists(p):
        return None
    rec = json.load(open(p)).get(workload)
    return None if rec is None else dict(rec, stale=rec.get("build") != build)


def measured_bound(counters, wkey):
    """The dominant kernel's binding pipe from its rocprof counters of THIS build: "lds" when the LDS array is
    busier (ROCm LdsUtil, SQ_LDS_IDX_ACTIVE) than the SIMDs issue VALU (VALUBusy), else "valu".  Falls back to
    dprf_amd/work.py's static BOUND when no current profile has the counters (source says which)."""
    from dprf_amd import work
    if counters and not counters.get("stale") and counters.get("lds_util") is not None and counters.get("valu_busy"):
        return ("lds" if counters["lds_util"] > counters["valu_busy"] else "valu"), "rocprof"
    return work.BOUND.get(wkey, "valu"), "model"


def latency_roof(wkey, per_gpu_rate):
    """R2-R4: the chain-latency bound (dprf_amd/work.py lds_latency_bound: 9 chains per CU at the unloaded chain
    latency tools/rc4_ksa_probe.hip measured) and the fraction of it this run reached, from its per-GPU wall rate"""
    from dprf_amd import work
    b = work.lds_latency_bound(wkey)
    if b is None:
        return None
    return {"bound_cand_per_s": b, "frac": per_gpu_rate / b, "chains_per_cu": work.RC4_CHAINS_PER_CU,
            "pass_ns_unloaded": work.RC4_PASS_NS_UNLOADED[wkey], "passes_per_candidate": work.RC4_PASSES[wkey],
            "source": work.RC4_LATENCY_SOURCE}


def issue_line(counters, wkey, pwlen):
    """The VALU issue accounting of the dominant kernel (round 6): the wave-instructions it executes per
    candidate lane and the SIMD cycles each takes (from the rocprof SQ pass of this build, profiles/pmc_valu.json), the
    algorithm's minimum instruction count (dprf_amd/work.py INSTR, the same dataflow functions as the slot floor) and
    their ratio instr_frac = floor / measured.  A kernel at instr_frac ~1 and ~3.9 cycles per instruction sits on the
    issue cadence of its own instruction mix: only fewer instructions could make it faster."""
    from dprf_amd import work
    floor = work.per_candidate(wkey, "instr", part="main", pwlen=pwlen)
    out = {"instr_floor": floor}
    if counters and counters.get("valu_instr_per_candidate"):
        ipc = counters["valu_instr_per_candidate"]
        out.update(instr_per_candidate=ipc, cycles_per_instr=counters.get("cycles_per_valu_instr"),
                   instr_frac=floor / ipc, source=counters.get("source"), stale=counters.get("stale"))
    return out


def compact_rocprof(rec):
    return None if not rec else {k: rec[k] for k in ROCPROF_KEYS if rec.get(k) is not None}


def compact_cpu(c):
    """A CPU baseline as the bench line carries it: the figures, one short sample description (the full records,
    with every leg's sample text, go to the stderr detail line)."""
    if not c:
        return c
    out = {k: c[k] for k in ("value", "unit", "cores", "kind", "nproc", "cpu_share") if k in c}
    out["sample"] = c.get("sample", "")[:160]
    for k in ("one_worker", "process_model_4"):
        if c.get(k):
            out[k] = {"value": c[k]["value"], "cores": c[k]["cores"]}
    return out


def device_balance(ctx):
    """Per-device split of the last library call (dprf_ctx_last_call_devices) when this process drives several
    GPUs through one context: candidates, launches, finish time, and the last device's finish over the mean."""
    devs = ctx.last_call_devices()
    if len(devs) < 2:
        return None
    fin = [d["finish_ms"] for d in devs]
    mean = sum(fin) / len(fin)
    return {"devices": devs, "last_over_mean": max(fin) / mean if mean > 0 else None}


def summarize(stats, wkey, world, dt, pwlen=None):
    from dprf_amd import work
    cands = sum(s["candidates"] for s in stats)
    launches = sum(s["launches"] for s in stats)
    kern_ms = sum(s["kernel_ms"] for s in stats)
    main_ms = sum(s["main_kernel_ms"] for s in stats)
    wall_ms = sum(s["wall_ms"] for s in stats)
    devs = max(1, max(s.get("devices", 1) for s in stats))
    avg_launch_ms = main_ms / max(1, launches)
    per_launch = cands / max(1, launches)
    floor = work.per_candidate(wkey, part="main", pwlen=pwlen)
    achieved = per_launch * floor / (avg_launch_ms / 1e3)
    spec = work.per_candidate(wkey, "spec", part="main")
    return {"cands": cands, "launches": launches, "kern_ms": kern_ms, "avg_launch_ms": avg_launch_ms,
            "per_launch": per_launch, "floor": floor, "achieved": achieved,
            "spec": spec, "achieved_spec": per_launch * spec / (avg_launch_ms / 1e3),
            # host time of the library calls not covered by device time (launch gaps, polling, hit merge)
            "call_overhead": 1.0 - kern_ms / max(1e-9, wall_ms * devs),
            "value": cands * world / dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="odt", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU candidates per step (default per workload)")
    ap.add_argument("--no-side", action="store_true", help="skip the per-format side measurements")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--no-cluster", action="store_true", help="skip the configs[4] server + GPU client leg")
    ap.add_argument("--cluster-candidates", type=int, default=12 << 20)
    ap.add_argument("--side-steps", type=int, default=5, help="timed steps of each per-format leg (1 warmup)")
    ap.add_argument("--stop-on-first", action="store_true",
                    help="time the product's early-stop rounds instead of full verification of every batch")
    args = ap.parse_args()

    rank, world, local = dist_env()
    import torch
    from dprf_amd import _lib, brute_force, work

    # Rehearsal knobs for the N>1 path on a 1-GPU box (never used by the driver): DPRF_BENCH_SAME_DEVICE=1
    # puts every rank on device 0 and DPRF_BENCH_BACKEND=gloo exchanges through CPU tensors (RCCL refuses two
    # ranks on one GPU).  DPRF_BENCH_FORCE_DIST=1 opens the process group even for a single torchrun rank, so
    # the RCCL init, barrier and MIN/MAX all-reduces run on a 1-GPU box.  The driver's runs use one GPU per
    # rank and RCCL.
    backend = os.environ.get("DPRF_BENCH_BACKEND", "nccl")
    if os.environ.get("DPRF_BENCH_SAME_DEVICE") == "1":
        local = 0
    dist = None
    if world > 1 or os.environ.get("DPRF_BENCH_FORCE_DIST") == "1":
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    # one process per GPU under torchrun (world = N); `--gpus N` without a launcher drives N GPUs from this
    # one process through one multi-device library context instead
    devices = [local]
    if world == 1 and args.gpus > 1:
        if os.environ.get("DPRF_BENCH_SAME_DEVICE") == "1":
            devices = [local] * args.gpus        # rehearsal: N library lanes (threads + streams) on one GPU
        else:
            devices = _lib.device_list()[:args.gpus]
        if len(devices) < args.gpus:
            raise SystemExit("--gpus %d: only %d gfx950 devices visible" % (args.gpus, len(devices)))

    def sync():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(torch.device("cuda", d))
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
    n_gpus = world * len(devices)

    cpu = None
    side_cpu = {}
    if rank == 0 and n_gpus == 1 and args.cpu_seconds > 0:
        cpu = cpu_baselines(fields, cs, pwlen, seconds=args.cpu_seconds)
        log("cpu baseline:", cpu)
        if not args.no_side:
            for name in SIDE_FORMATS:
                if name == args.workload:
                    continue
                sn, scs, spl, _, _, _ = WORKLOADS[name]
                sf = quiet_fields(brute_force, S[sn]["stream"])
                # every format gets brute_force.py's own structure (4 processes, one Popen of the reference verifier
                # per candidate), 1 worker and all cores of the job's share (round 5)
                side_cpu[name] = cpu_baselines(sf, scs, spl, seconds=min(1.0, args.cpu_seconds))

    ctx = _lib.Context(fields, devices=devices)
    B = args.batch or B
    dt, stats, lowest, pwlen = run_workload(args.workload, ctx, rank, world, args.steps, args.warmup, sync,
                                            allreduce_min, B, ndev=len(devices), stop_on_first=args.stop_on_first)
    dt_max = allreduce_max(dt)
    m = summarize(stats, wkey, world, dt_max, pwlen)
    peak = work.PEAK_LANE_INSTR_PER_S
    build = _lib.build_id()
    pmc = os.path.join(HERE, "profiles", "pmc_traffic.json")
    traffic, traffic_rec = launch_traffic(pmc, args.workload, m["per_launch"], build)
    counters = pmc_summary(args.workload, build)
    balance = device_balance(ctx)

    side = {}
    if not args.no_side:
        for name in SIDE_FORMATS:
            if name == args.workload:
                continue
            sn, scs, spl, sB, skey, sdesc = WORKLOADS[name]
            sf = quiet_fields(brute_force, S[sn]["stream"])
            sctx = _lib.Context(sf, devices=devices)
            sdt, sst, _, spl = run_workload(name, sctx, rank, world, args.side_steps, 1, sync, allreduce_min,
                                            ndev=len(devices))
            sdt = allreduce_max(sdt)
            sm = summarize(sst, skey, world, sdt, spl)
            per_gpu = sm["value"] / world / max(1, len(devices))
            pc = pmc_summary(name, build)
            side[name] = {"value": sm["value"], "unit": "candidates/s", "kernel": sctx.kernel, "config": sdesc,
                          "pwlen": spl, "bound": measured_bound(pmc_summary(name, build), skey)[0],
                          "steps": args.side_steps, "avg_launch_ms": sm["kern_ms"] / max(1, sm["launches"]),
                          "dominant_avg_ms": sm["avg_launch_ms"], "candidates_per_launch": sm["per_launch"],
                          # the larger of the launch-time and the wall-time figure: R2-R4 launches overlap on two
                          # streams (a launch's event time then includes its neighbour's), other formats' do not
                          "valu_floor_frac": max(sm["per_launch"] * work.per_candidate(skey, pwlen=spl)
                                                 / (sm["kern_ms"] / max(1, sm["launches"]) / 1e3) / peak,
                                                 per_gpu * work.per_candidate(skey, pwlen=spl) / peak),
                          # SURVEY 8(d)'s spec-level VALU ops per candidate over the same peak, same time base; its LDS
                          # lane-operations against one LDS per CU (round 6: the LDS ops no longer counted as VALU)
                          "spec_frac": max(sm["per_launch"] * work.per_candidate(skey, "spec")
                                           / (sm["kern_ms"] / max(1, sm["launches"]) / 1e3) / peak,
                                           per_gpu * work.per_candidate(skey, "spec") / peak),
                          "lds_spec_frac": work.lds_spec_frac(skey, per_gpu),
                          "issue": issue_line(pc, skey, spl),
                          "call_overhead": sm["call_overhead"]}
            if skey in work.SPEC_EFFECTIVE:
                side[name]["spec_effective"] = True
            lat = latency_roof(skey, per_gpu)
            if lat:
                side[name]["limiter"] = "lds-latency"
                side[name]["lds_latency"] = lat
            if skey in work.LDS_CYCLES:             # RC4 formats: the modelled LDS-array share (~ rocprof LdsUtil)
                side[name]["lds_cycle_frac"] = work.lds_frac(
                    skey, sm["per_launch"] / (sm["kern_ms"] / max(1, sm["launches"]) / 1e3))
            if pc:
                side[name]["rocprof"] = compact_rocprof(pc)
            tr, trec = launch_traffic(pmc, name, sm["per_launch"], build)
            if tr is not None:
                side[name]["traffic_bytes_per_launch"] = tr
                side[name]["traffic_source"] = {k: trec.get(k) for k in ("source", "build", "stale")}
            if name in side_cpu:
                side[name]["cpu_baseline"] = compact_cpu(side_cpu[name])
            sctx.close()

    cluster = None
    if rank == 0 and n_gpus == 1 and not args.no_side and not args.no_cluster:
        # configs[4]: server + GPU clients over TCP on this box (2 client processes on this GPU hide each
        # other's request/parse gaps), Office test document, -pr 8 order, 2^20-candidate payloads
        sys.path.insert(0, os.path.join(HERE, "tools"))
        import bench_cluster
        try:
            cluster = bench_cluster.run(gpus=1, clients_per_gpu=2, payload=1 << 20,
                                        candidates=args.cluster_candidates, workload="office",
                                        timeout=180, devices=[local])
            cluster.pop("clients_detail", None)
        except Exception as ex:   # the leg is reported, never fatal to the headline line
            cluster = {"error": repr(ex)}

    if rank == 0:
        bound, bound_src = measured_bound(counters, wkey)
        roof = {"bound": bound, "bound_source": bound_src, "achieved": m["achieved"] / 1e12, "peak": peak / 1e12,
                "unit": "T VALU lane-slots/s (gfx950 issue-slot floor of the algorithm)",
                "frac": m["achieved"] / peak, "valu_floor_frac": m["achieved"] / peak,
                # the same kernel time against SURVEY 8(d)'s spec-level op count (2-input ops, 3-input = 2)
                "spec_frac": m["achieved_spec"] / peak, "spec_achieved": m["achieved_spec"] / 1e12,
                "lds_spec_frac": work.lds_spec_frac(wkey, m["value"] / world / max(1, len(devices))),
                "issue": issue_line(counters, wkey, pwlen),
                "traffic": traffic,
                "kernel": DOMINANT.get(ctx.kernel, ctx.kernel),
                "kernel_avg_ms": m["avg_launch_ms"], "candidates_per_launch": m["per_launch"],
                "floor_instr_per_candidate": m["floor"],
                "all_kernels_avg_ms": m["kern_ms"] / max(1, m["launches"]),
                "all_kernels_frac": m["cands"] * work.per_candidate(wkey) / (m["kern_ms"] / 1e3) / peak,
                "spec_ops_per_candidate": work.per_candidate(wkey, "spec"),
                "lds_cycle_frac": work.lds_frac(wkey, m["per_launch"] / (m["avg_launch_ms"] / 1e3)),
                "call_overhead": m["call_overhead"]}
        if wkey in work.SPEC_EFFECTIVE:
            roof["spec_effective"] = True
        lat = latency_roof(wkey, m["value"] / world / max(1, len(devices)))
        if lat:             # R2-R4: the chain-latency bound the design can approach (work.py); frac stays the VALU one
            roof["lds_latency"] = lat
            roof["limiter"] = "lds-latency (model: 9 chains/CU at the unloaded chain latency, tools/rc4_ksa_probe.hip)"
        if traffic_rec:
            roof["traffic_source"] = {k: traffic_rec.get(k) for k in ("source", "build", "stale", "fetch_bytes",
                                                                      "write_bytes", "bytes_per_candidate")}
        if counters:
            roof["valu_busy"] = counters.get("valu_busy")
            roof["valu_utilization"] = counters.get("valu_utilization")
            roof["rocprof"] = compact_rocprof(counters)
        out = {
            "metric": METRIC,
            "value": m["cands"] * world / dt_max,
            "unit": "candidates/s",
            "n_gpus": n_gpus,
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
                       "batch_per_gpu": B, "kernel": ctx.kernel, "build": build,
                       "parallelism": "keyspace shards x%d (%s)" % (
                           n_gpus, "one process per GPU" if dist else
                           "one process, %d-device library context" % len(devices))},
            "roofline": roof,
            "cpu_baseline": compact_cpu(cpu),
            "per_format": side,
            "cluster": None if cluster is None else {k: v for k, v in cluster.items() if not isinstance(v, (list, dict))},
            "lowest_hit_index": None if lowest is None or lowest >= (1 << 62) else lowest,
        }
        if balance:
            out["device_balance"] = balance
        # every workload's figure in a few hundred bytes at the END of the line, so that a log tail shows all of
        # them (the 16 KB driver tail started inside the per-format CPU samples)
        # kernel_ms is per launch; the launch size ("cand") lets it be compared per candidate with a profile whose
        # rate-driven launches differ in size (R2-R4: launches also overlap on two streams)
        def cpu_short(c):
            """the CPU figures of a leg, cand/s: all cores of the share / 1 worker / brute_force.py's 4 processes"""
            if not c:
                return None
            g = lambda k: round(c[k]["value"], 1) if c.get(k) else None
            return {"all": round(c["value"], 1), "cores": c.get("cores"), "one": g("one_worker"),
                    "pm4": g("process_model_4")}

        def issue_short(i):
            """instructions per candidate, cycles per instruction, instruction floor / measured"""
            r = lambda x, n: None if x is None else round(x, n)
            return {"instr_per_candidate": r(i.get("instr_per_candidate"), 1), "cycles_per_instr": r(i.get("cycles_per_instr"), 3),
                    "instr_frac": r(i.get("instr_frac"), 4)}

        summ = {args.workload: dict({"value": out["value"], "valu_floor_frac": roof["valu_floor_frac"],
                                     "spec_frac": roof["spec_frac"], "lds_spec_frac": roof["lds_spec_frac"],
                                     "kernel_ms": m["avg_launch_ms"], "cand": int(m["per_launch"]), "steps": args.steps,
                                     "cpu": cpu_short(cpu)}, **issue_short(roof["issue"]))}
        if roof.get("lds_latency"):
            summ[args.workload]["lds_latency_frac"] = roof["lds_latency"]["frac"]
        for name, v in side.items():
            summ[name] = dict({"value": v["value"], "valu_floor_frac": v["valu_floor_frac"], "spec_frac": v["spec_frac"],
                               "lds_spec_frac": v["lds_spec_frac"], "kernel_ms": v["dominant_avg_ms"],
                               "cand": int(v["candidates_per_launch"]), "steps": v["steps"],
                               "cpu": cpu_short(side_cpu.get(name))}, **issue_short(v["issue"]))
            if v.get("spec_effective"):
                summ[name]["spec_effective"] = True
            if v.get("lds_latency"):
                summ[name]["lds_latency_frac"] = v["lds_latency"]["frac"]
        if cluster and cluster.get("value") is not None:
            summ["cluster"] = {"value": cluster.get("value"), "clients": cluster.get("clients")}
        out["summary"] = {"build": build, "workloads": summ}
        # the full records (every CPU leg's sample text, whole rocprof summaries, cluster details) on stderr
        log("bench detail: " + json.dumps({"cpu_baseline": cpu, "per_format_cpu": side_cpu, "cluster": cluster,
                                           "rocprof": counters}))
        print(json.dumps(out), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

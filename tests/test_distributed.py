"""Multi-rank path on CPU (gloo, world_size 2): the bench's per-rank keyspace shards tile each step's
block exactly, and the RCCL-side exchange (all-reduce MIN of the lowest hit index, MAX of the time)
behaves as the GPU run relies on.  The same code runs over nccl (RCCL) on the MI355X node."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    B, space = 1000, 62 ** 3
    starts = []
    for step in range(5):
        s, n = bench.shard(step, rank, world, B, space)
        starts.append((s, n))
        # pretend rank r found hits at these indices; the job's answer is the global lowest
        first = torch.tensor([s + 17 * (rank + 1) if step == 3 else (1 << 62)], dtype=torch.int64)
        dist.all_reduce(first, op=dist.ReduceOp.MIN)
        if step == 3:
            q.put(("min", rank, int(first.item())))
    t = torch.tensor([0.5 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    q.put(("shards", rank, starts, float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


class OracleCtx:
    """Stand-in for _lib.Context on CPU (test infrastructure): the oracle's verdicts over the same range."""

    def __init__(self, stream):
        import pyoracle
        self.c = pyoracle.Ctx(stream)

    def search_range(self, cs, pwlen, start, n, stop_on_first=False, cap=1 << 16):
        hits, nh = self.c.search_range(cs, pwlen, start, n, nthreads=2)
        return hits[:cap], nh, {"candidates": n, "wall_ms": 1.0, "launches": 1, "kernel_ms": 1.0,
                                "main_kernel_ms": 1.0, "devices": 1}


def _bench_worker(rank, world, port, q):
    """bench.run_workload itself on two gloo ranks with an oracle-backed context: the shards, the per-round
    call (brute_force.search_round) and the MIN exchange of a REAL hit (PDF R5 doc, password 'cat')."""
    import sys
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(here, "oracle"))
    import json
    import bench
    streams = json.load(open(os.path.join(here, "tests", "golden", "streams.json")))
    bench.WORKLOADS["test_r5"] = ("pdf_synth_r5_cat", bench.LOWER, 3, 1000, "pdf_r5", "gloo test")

    def amin(v):
        t = torch.tensor([v], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    ctx = OracleCtx(streams["pdf_synth_r5_cat"]["stream"])
    dt, stats, lowest, pwlen = bench.run_workload("test_r5", ctx, rank, world, 3, 0, dist.barrier, amin)
    q.put((rank, lowest, pwlen, [s["candidates"] for s in stats]))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_run_workload_two_ranks_min_of_a_real_hit():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    [p.join(120) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    res = sorted(q.get(timeout=5) for _ in range(world))
    want = 2 * 676 + 0 * 26 + 19          # "cat" in lowercase^3 product order, verified by rank 1 in step 0
    assert [r[1] for r in res] == [want, want]
    assert all(r[2] == 3 and r[3] == [1000, 1000, 1000] for r in res)


def test_two_rank_shards_and_allreduce():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    [p.start() for p in procs]
    [p.join(120) for p in procs]
    assert all(p.exitcode == 0 for p in procs)
    msgs = [q.get(timeout=5) for _ in range(2 * world)]
    shards = {m[1]: m[2] for m in msgs if m[0] == "shards"}
    mins = [m[2] for m in msgs if m[0] == "min"]
    tmax = [m[3] for m in msgs if m[0] == "shards"]
    import bench
    for step in range(5):
        pieces = sorted(shards[r][step] for r in range(world))
        assert pieces[0][0] + pieces[0][1] == pieces[1][0], "ranks' slices must be adjacent"
        assert pieces[0][0] == (step * world * 1000) % (62 ** 3 - 1000)
    s3 = [shards[r][3][0] for r in range(world)]
    assert mins == [min(s + 17 * (r + 1) for r, s in enumerate(s3))] * world
    assert tmax == [1.5, 1.5]


def test_brute_force_rounds_are_sized_by_time():
    """brute_force's range rounds: the first is FIRST_ROUND candidates, later ones ~ROUND_SECONDS at the
    measured rate, never past the end of the keyspace (the library splits each round over the devices)."""
    from dprf_amd import brute_force as bf
    assert bf.next_round(0.0, 1 << 40) == bf.FIRST_ROUND
    assert bf.next_round(1e9, 1 << 40) == int(1e9 * bf.ROUND_SECONDS)
    assert bf.next_round(10.0, 1 << 40) == bf.FIRST_ROUND
    assert bf.next_round(1e9, 12345) == 12345


def test_small_keyspace_shards_stay_disjoint_at_eight_ranks():
    """Office -pr 4 is one batch: at N > 1 bench.run_workload moves to the next length so the ranks'
    slices of every step are disjoint instead of all ranks verifying the same candidates."""
    import bench

    seen = {}

    class FakeCtx:
        def __init__(self, rank):
            self.rank = rank

        def search_range(self, cs, pwlen, start, n, stop_on_first=False, cap=1 << 16):
            seen.setdefault(pwlen, []).append((start, n))
            return [], 0, {"candidates": n, "wall_ms": 1.0}

    world = 8
    for rank in range(world):
        _, _, _, pwlen = bench.run_workload("office", FakeCtx(rank), rank, world, 2, 1, lambda: None, lambda v: v)
        assert pwlen == 5
    spans = sorted(seen[5])
    assert len(spans) == 3 * world
    for (s0, n0), (s1, _) in zip(spans, spans[1:]):
        assert s0 + n0 <= s1
    assert all(n == 26 ** 4 for _, n in spans)

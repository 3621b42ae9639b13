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


def test_brute_force_round_slices_tile_the_block():
    """brute_force's in-process multi-device rounds: every device gets a contiguous slice of the round's
    block and the slices tile it (the lowest hit of a round is then the lowest overall)."""
    from dprf_amd import brute_force as bf
    for ndev in (1, 2, 3, 8):
        for done, block in ((0, 1000), (5000, 7), (123, 1 << 20)):
            sl = bf._round_slices(done, block, ndev)
            assert sl[0][0] == done
            for (a, n), (b, _) in zip(sl, sl[1:]):
                assert a + n == b
            assert sum(n for _, n in sl) == block


def test_small_keyspace_shards_stay_disjoint_at_eight_ranks():
    """Office -pr 4 is one batch: at N > 1 bench.run_workload moves to the next length so the ranks'
    slices of every step are disjoint instead of all ranks verifying the same candidates."""
    import bench

    seen = {}

    class FakeCtx:
        def __init__(self, rank):
            self.rank = rank

        def search_range(self, cs, pwlen, start, n):
            seen.setdefault(pwlen, []).append((start, n))
            return [], 0, {"candidates": n}

    world = 8
    for rank in range(world):
        _, _, _, pwlen = bench.run_workload("office", FakeCtx(rank), rank, world, 2, 1, lambda: None, lambda v: v)
        assert pwlen == 5
    spans = sorted(seen[5])
    assert len(spans) == 3 * world
    for (s0, n0), (s1, _) in zip(spans, spans[1:]):
        assert s0 + n0 <= s1
    assert all(n == 26 ** 4 for _, n in spans)

"""World-size-2 gloo test of the window sharding and the final consensus
gather used by bench.py --gpus N; runs on CPU."""
import os
import socket

import torch.distributed as dist
import torch.multiprocessing as mp

from claragenomicsanalysis_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard.window_range(rank, 5)
    cons = ["W%d_%s" % (first + i, "ACGT" * (first + i)) for i in range(n)]
    got = shard.gather_consensus(cons, 200)
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_window_ranges_disjoint():
    seen = set()
    for r in range(8):
        first, n = shard.window_range(r, 125000)
        rng = set(range(first, first + n))
        assert not (rng & seen)
        seen |= rng
    assert min(seen) == 1 and max(seen) == 1000000


def test_pack_roundtrip():
    s = ["", "A", "ACGT" * 10]
    assert shard.unpack_strings(shard.pack_strings(s, 64)) == s


def test_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert got == ["W%d_%s" % (s, "ACGT" * s) for s in range(1, 11)]


def test_shard_windows_balance_and_cover():
    import random
    rng = random.Random(3)
    groups = [["A" * rng.randint(100, 12000)] * rng.randint(2, 40) for _ in range(997)]
    for world in (1, 2, 3, 8):
        shards = shard.shard_windows(groups, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(groups)))
        counts = [len(s) for s in shards]
        assert max(counts) - min(counts) <= 1
        cost = [sum(shard.window_cost(groups[i]) for i in s) for s in shards]
        assert max(cost) <= 1.05 * min(cost)
    assert shard.shard_windows([], 4) == [[], [], [], []]


def _sharded_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    groups = [["ACGT" * (i % 5 + 1)] * (i % 3 + 2) for i in range(7)]
    shards = shard.shard_windows(groups, world)
    mine = ["C%d" % i for i in shards[rank]]  # stand-in for this rank's consensus strings
    got = shard.gather_sharded(mine, shards, 16)
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_gather_sharded_restores_window_order():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert got == ["C%d" % i for i in range(7)]

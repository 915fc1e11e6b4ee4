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


def _stream_worker(rank, world, port, out):
    # config E's rank partition and gather (bench.py bench_stream): rank r owns
    # seeds stream_window_range(r, steps, per_step); its consensus rows
    # [len | status | bytes] are gathered to rank 0 in rank order
    import numpy as np
    from claragenomicsanalysis_amd import synth
    from oracle import oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = shard.stream_window_range(rank, 2, 3)
    wins = synth.poa_windows(first, n, 120, 5, 6, 6, 6)
    cons, status, cells, _ = oracle.poa_batch(wins, max_nodes=600, max_consensus=400, max_seqs=5)
    rows = np.zeros((n, 8 + 400), np.uint8)
    for i, c in enumerate(cons):
        rows[i, :4] = np.frombuffer(np.int32(len(c)).tobytes(), np.uint8)
        rows[i, 4:8] = np.frombuffer(np.int32(status[i]).tobytes(), np.uint8)
        rows[i, 8:8 + len(c)] = np.frombuffer(c.encode(), np.uint8)
    got = shard.gather_rows(rows)
    if rank == 0:
        out.put(got)
    dist.barrier()
    dist.destroy_process_group()


def test_stream_partition_and_gather_world2_gloo():
    import numpy as np
    from claragenomicsanalysis_amd import synth
    from oracle import oracle
    assert [shard.stream_window_range(r, 20, 6250) for r in range(8)] == [(1 + 125000 * r, 125000)
                                                                          for r in range(8)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stream_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # the gathered rows are seeds 1..12 in order, as one rank would have computed them
    wins = synth.poa_windows(1, 12, 120, 5, 6, 6, 6)
    cons, status, _, _ = oracle.poa_batch(wins, max_nodes=600, max_consensus=400, max_seqs=5)
    assert got.shape == (12, 408)
    lens = got[:, :4].copy().view(np.int32).ravel()
    st = got[:, 4:8].copy().view(np.int32).ravel()
    assert st.tolist() == [int(s) for s in status]
    assert [got[i, 8:8 + lens[i]].tobytes().decode() for i in range(12)] == cons

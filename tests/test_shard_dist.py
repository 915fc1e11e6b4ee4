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

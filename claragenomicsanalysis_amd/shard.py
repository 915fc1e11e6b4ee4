"""Window sharding and the final consensus gather.

Windows are independent, so each rank (one process per GPU) owns a disjoint
window range and runs its own batch; no data moves between ranks while
windows are processed.  After that, rank 0 gathers every rank's consensus
strings once: the strings are packed as [len:int32 | bytes] rows of a fixed
width into one uint8 tensor per rank and collected with
``torch.distributed.gather`` (RCCL over xGMI with the nccl backend on GPUs,
gloo on CPUs).  This generalises the reference's one-batch-per-device
driver (cudapoa/src/multi_batch.hpp:36-170).
"""
import numpy as np
import torch
import torch.distributed as dist


def window_range(rank, windows_per_rank):
    """First synthetic seed and count of a rank's windows (seeds 1..N overall)."""
    return 1 + rank * windows_per_rank, windows_per_rank


def pack_strings(strings, width):
    buf = np.zeros((len(strings), width + 4), np.uint8)
    for i, s in enumerate(strings):
        b = s.encode() if isinstance(s, str) else bytes(s)
        if len(b) > width:
            raise ValueError("string %d longer than the gather width %d" % (i, width))
        buf[i, :4] = np.frombuffer(np.int32(len(b)).tobytes(), np.uint8)
        buf[i, 4:4 + len(b)] = np.frombuffer(b, np.uint8)
    return buf


def unpack_strings(buf):
    out = []
    for row in buf:
        n = int(np.frombuffer(row[:4].tobytes(), np.int32)[0])
        out.append(row[4:4 + n].tobytes().decode())
    return out


def gather_consensus(strings, width, device=None):
    """Gather every rank's strings to rank 0 (rank order); other ranks get None.

    All ranks must pass the same number of strings and the same width.
    """
    world = dist.get_world_size()
    rank = dist.get_rank()
    t = torch.from_numpy(pack_strings(strings, width))
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    if rank != 0:
        return None
    out = []
    for p in parts:
        out.extend(unpack_strings(p.cpu().numpy()))
    return out


def gather_rows(rows, device=None):
    """Gather every rank's uint8 row array (same shape on every rank) to rank 0
    in rank order: returns the concatenated numpy array on rank 0, None
    elsewhere.  Used for config E's packed [len | status | consensus] rows,
    so no per-window Python strings are built on either side."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    t = torch.from_numpy(np.ascontiguousarray(rows, dtype=np.uint8))
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    if rank != 0:
        return None
    return np.concatenate([p.cpu().numpy() for p in parts], axis=0)


def stream_window_range(rank, steps, windows_per_step):
    """Config E: first seed and count of a rank's windows (steps x windows_per_step
    per rank, seeds 1 + rank * count ...; 20 x 6250 = 125k per rank)."""
    n = steps * windows_per_step
    return 1 + rank * n, n


def window_cost(group):
    """DP cells of a window up to a constant: (reads - 1) x (longest read)^2
    (each read is aligned to a graph about as long as the reads)."""
    lens = [len(r) for r in group]
    if len(lens) < 2:
        return 0
    m = max(lens)
    return (len(lens) - 1) * m * m


def shard_windows(groups, world_size):
    """Window indices per rank for real (uneven) data, SURVEY.md 8(e): the
    windows are ordered by cost and dealt in snake order (0..N-1, N-1..0, ...),
    so every rank gets a similar number of windows and of DP cells.  The
    reference balances nothing across devices (main.cu:491-513 hands out
    whole batches); this is the per-rank analogue of get_multi_batch_sizes'
    size binning (utils.cu:24-138).  Each rank's list is ascending."""
    if world_size < 1:
        raise ValueError("world_size must be at least 1")
    order = sorted(range(len(groups)), key=lambda i: (-window_cost(groups[i]), i))
    shards = [[] for _ in range(world_size)]
    for k, i in enumerate(order):
        cyc, pos = divmod(k, world_size)
        shards[pos if cyc % 2 == 0 else world_size - 1 - pos].append(i)
    return [sorted(s) for s in shards]


def gather_sharded(strings, shards, width, device=None):
    """Gather every rank's strings (one per window of its shard, in shard
    order) to rank 0 and return them in the original window order; other
    ranks get None.  Shards may differ in size by one window."""
    n = max(len(s) for s in shards)
    rank = dist.get_rank()
    if len(strings) != len(shards[rank]):
        raise ValueError("rank %d passes %d strings for %d windows" % (rank, len(strings), len(shards[rank])))
    got = gather_consensus(list(strings) + [""] * (n - len(strings)), width, device)
    if got is None:
        return None
    out = [None] * sum(len(s) for s in shards)
    for r, s in enumerate(shards):
        for j, idx in enumerate(s):
            out[idx] = got[r * n + j]
    return out

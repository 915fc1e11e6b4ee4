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

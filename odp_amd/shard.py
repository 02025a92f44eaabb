"""Multi-GPU sharding of a packet batch.

Packets are independent, so a batch splits by packet index range. Each rank
classifies its shard against its own copy of the table snapshot. There is no
collective on the data path. The reference keeps per-CoS and pktio counters
globally (``odp_cls_cos_stats``, odp_classification.c:1621-1622,1697-1698;
loop.c:304-374), so a multi-GPU job sums its counter blocks once per batch
with one all-reduce. The collective backend is RCCL ("nccl") on GPUs, gloo in
the CPU tests.
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total, rank, world):
    """[start, start + count) of packet indices owned by ``rank``: contiguous
    ranges, sizes differing by at most one, covering 0..n_total exactly once."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(n_total), int(world))
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def reduce_counters(stats, dist, device=None):
    """Sum a u64 counter block (``ODPG_STATS_WORDS`` words) over all ranks.

    ``dist`` is ``torch.distributed`` (initialised) or None for one rank.
    Values travel as int64; counters never reach 2^63."""
    stats = np.asarray(stats, dtype=np.uint64)
    if dist is None:
        return stats
    import torch
    t = torch.from_numpy(stats.astype(np.int64))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(np.uint64)


def max_over_ranks(x, dist, device=None):
    """Max of a float over ranks (the bench's timed wall clock)."""
    if dist is None:
        return float(x)
    import torch
    t = torch.tensor([float(x)], dtype=torch.float64)
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_verdicts(out, dist, n_total, world, device=None):
    """Concatenate every rank's u32 verdict shard on all ranks (tests and
    host-side enqueue; not on the device-resident metric's path)."""
    out = np.asarray(out, dtype=np.uint32)
    if dist is None:
        return out
    import torch
    counts = [shard_range(n_total, r, world)[1] for r in range(world)]
    mx = max(counts)
    buf = np.zeros(mx, dtype=np.int64)
    buf[:len(out)] = out.astype(np.int64)
    t = torch.from_numpy(buf)
    if device is not None:
        t = t.to(device)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return np.concatenate([p.cpu().numpy()[:c].astype(np.uint32) for p, c in zip(parts, counts)])


def broadcast_bytes(data, dist, device=None, src=0):
    """Broadcast a byte string from ``src`` (the compiled table image,
    odpg_rules_compile: once per table generation); other
    ranks pass None and receive it."""
    if dist is None:
        return data
    import torch
    n = torch.tensor([len(data) if data is not None else 0], dtype=torch.int64)
    if device is not None:
        n = n.to(device)
    dist.broadcast(n, src)
    size = int(n.item())
    if data is not None and dist.get_rank() == src:
        buf = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    else:
        buf = torch.zeros(size, dtype=torch.uint8)
    if device is not None:
        buf = buf.to(device)
    dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def scatter_shards(whole, shard, dist, src=0):
    """One batch that originates on rank ``src``'s GPU, split by packet range
    over the ranks (SURVEY §8(e) "scatter over xGMI"): ``whole`` is a
    [world * per_rank, stride] uint8 tensor on ``src`` (None elsewhere),
    ``shard`` this rank's [per_rank, stride] receive tensor. Equal shards."""
    world = dist.get_world_size()
    parts = list(whole.chunk(world)) if dist.get_rank() == src else None
    dist.scatter(shard, parts, src=src)
    return shard


def gather_to_root(part, dist, dst=0):
    """Every rank's verdict shard (equal sizes) concatenated on ``dst``
    (grouped send/recv to the root); None on other ranks."""
    import torch
    world = dist.get_world_size()
    if dist.get_rank() == dst:
        parts = [torch.empty_like(part) for _ in range(world)]
        dist.gather(part, parts, dst=dst)
        return torch.cat(parts)
    dist.gather(part, None, dst=dst)
    return None

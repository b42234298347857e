"""Multi-GPU sharding of the query batch: every query is independent, so the
index is replicated on each GPU and queries are split into contiguous ranges; the only exchange is
gathering fixed-size per-rank results to rank 0 for output (indices/distances/SW scores), off the
hot path. gather_rows is the host-side form over a torch.distributed group (gloo: the CPU tests);
device-resident rows go over RCCL from C++ (drm_comm_gather_rows, executor.Comm)."""
import numpy as np


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of rank `rank` out of `world` for n queries: [r*n/G, (r+1)*n/G)."""
    lo = (rank * n) // world
    hi = ((rank + 1) * n) // world
    return lo, hi


def gather_rows(arr, n_total, rank, world, dist):
    """Gather per-rank row blocks [lo:hi) of a [n_total, ...] result to rank 0 (returns the full
    array on rank 0, None elsewhere). Uses all_gather on padded equal-size blocks."""
    import torch
    lo, hi = shard_range(n_total, rank, world)
    rows = max(shard_range(n_total, r, world)[1] - shard_range(n_total, r, world)[0] for r in range(world))
    a = np.ascontiguousarray(arr)
    assert a.shape[0] == hi - lo
    flat = a.view(np.uint8).reshape(a.shape[0], -1)
    width = flat.shape[1] if a.shape[0] else int(np.prod(a.shape[1:], dtype=np.int64)) * a.dtype.itemsize
    buf = np.zeros((rows, width), dtype=np.uint8)
    buf[:flat.shape[0]] = flat
    t = torch.from_numpy(buf)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    if rank != 0:
        return None
    parts = []
    for r in range(world):
        l, h = shard_range(n_total, r, world)
        parts.append(outs[r].numpy()[: h - l])
    full = np.concatenate(parts, axis=0)
    return full.view(a.dtype).reshape((n_total,) + a.shape[1:])

"""Multi-GPU tracing across processes (one process per GPU, torch.distributed).

Rays are independent, so a bundle shards by contiguous index ranges with NO data-path collective:
every rank traces ``rays[lo:hi]`` on its own GPU.  A collective is used only when the
caller asks for the whole history on every rank (``gather=True``, an all-gather over the shards) --
the reference has no such step; it exists for convenience, not for the trace.

Within ONE process, ``System.ray_trace(..., devices=[...])`` shards over several GPUs with one host
thread per device inside librtpb.so instead.
"""
import numpy as np


def shard_bounds(n, rank, world):
    """Contiguous shard [lo, hi) of n rays for ``rank`` of ``world`` (same split as rtpb_trace_host)."""
    return n * rank // world, n * (rank + 1) // world


def trace_sharded(system, rays, initial_material, final_material, *, group=None, gather=False, trace_fn=None,
                  **trace_kwargs):
    """Trace this rank's shard of ``rays`` (N, 8) and return ``(lo, hi, history_shard)``; with
    ``gather=True`` return the full (P, N, 8) history on every rank instead (all_gather over ranks).

    ``trace_fn(system, rays_shard, m0, m1, **kw)`` defaults to ``system.ray_trace`` (the GPU path)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    n = rays.shape[0]
    lo, hi = shard_bounds(n, rank, world)
    fn = trace_fn or (lambda s, r, a, b, **kw: s.ray_trace(r, a, b, **kw))
    local = fn(system, rays[lo:hi], initial_material, final_material, **trace_kwargs)
    if not gather:
        return lo, hi, local
    is_np = isinstance(local, np.ndarray)
    t = torch.from_numpy(np.ascontiguousarray(local)) if is_np else local
    P = t.shape[0]
    sizes = [shard_bounds(n, r, world) for r in range(world)]
    maxlen = max(b - a for a, b in sizes)
    pad = torch.full((P, maxlen, 8), float("nan"), dtype=t.dtype, device=t.device)
    pad[:, : t.shape[1]] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    full = torch.cat([b[:, : (hi_ - lo_)] for b, (lo_, hi_) in zip(bufs, sizes)], dim=1)
    return full.numpy() if is_np else full

"""Multi-GPU data parallelism over independent stereo pairs.

One process per GPU.  A batch of B frame pairs is partitioned into contiguous
shards (pair i -> rank i at B = N); every rank block-matches its own pairs with
no data-path collective, and rank 0 collects the u8 disparity maps with one
gather (RCCL over xGMI on MI355X, gloo in the CPU tests).  Distance maps are a
pure function of the disparity map (a 256-entry table), so only the 1 B/pixel
disparity crosses the fabric; rank 0 can expand it with disparity_to_distance.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def pair_range(batch: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [start, stop) of a batch of `batch` pairs for `rank` of `world`."""
    if world < 1 or not 0 <= rank < world or batch < 0:
        raise ValueError("bad batch / rank / world")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_disparity(local: torch.Tensor, batch: int, dst: int = 0, group=None, async_op: bool = False,
                     recv: list | None = None, concat: bool = True):
    """Gather every rank's (n_local, H, W) u8 maps into a (batch, H, W) tensor on `dst`.

    Shards may be uneven; each rank pads to the largest shard so one gather
    call moves everything.  `recv` (dst only): reusable receive buffers, one
    (max_shard, H, W) tensor per rank (a steady-state loop allocates nothing).
    `concat=False` returns the per-rank shards as a list of views instead of
    copying them into one tensor.  Returns the result on dst (None elsewhere),
    or, with async_op, a handle whose wait() returns it.
    """
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    start, stop = pair_range(batch, rank, world)
    if local.shape[0] != stop - start:
        raise ValueError(f"rank {rank} holds {local.shape[0]} maps, shard is {stop - start}")
    width = max(pair_range(batch, r, world)[1] - pair_range(batch, r, world)[0] for r in range(world))
    send = local
    if local.shape[0] < width:
        pad = torch.zeros((width - local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                          device=local.device)
        send = torch.cat([local, pad], 0)
    bufs = None
    if rank == dst:
        bufs = recv if recv is not None else [torch.empty_like(send) for _ in range(world)]
        if len(bufs) != world or any(b.shape != send.shape or b.dtype != send.dtype for b in bufs):
            raise ValueError("recv must hold one buffer per rank shaped like the padded shard")
    work = dist.gather(send.contiguous(), bufs, dst=dst, group=group, async_op=async_op)

    def assemble():
        if rank != dst:
            return None
        parts = []
        for r in range(world):
            s, e = pair_range(batch, r, world)
            parts.append(bufs[r][: e - s])
        return torch.cat(parts, 0) if concat else parts

    if async_op:
        class _Pending:
            def wait(self_inner):
                work.wait()
                return assemble()
        return _Pending()
    return assemble()

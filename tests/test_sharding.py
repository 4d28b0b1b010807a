"""N > 1 path on CPU: pair sharding and the rank-0 disparity gather over gloo
(world size 2), the same code bench.py runs over RCCL on the MI355X node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from unsynchronized_stereo_vision_proj325_amd.sharding import gather_disparity, pair_range


def test_pair_range_partitions():
    for batch in range(0, 20):
        for world in range(1, 9):
            spans = [pair_range(batch, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == batch
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [e - s for s, e in spans]
            assert max(sizes) - min(sizes) <= 1
    assert pair_range(8, 3, 8) == (3, 4)  # config D: pair i -> GPU i
    with pytest.raises(ValueError):
        pair_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, batch, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s, e = pair_range(batch, rank, world)
        # each pair's map is filled with its global pair index (and a ramp) so order is checkable
        local = torch.stack([(torch.arange(6 * 10, dtype=torch.int32).reshape(6, 10) + 7 * i) % 256
                             for i in range(s, e)]).to(torch.uint8) if e > s else \
            torch.empty((0, 6, 10), dtype=torch.uint8)
        out = gather_disparity(local, batch)
        pend = gather_disparity(local, batch, async_op=True).wait()
        width = max(pair_range(batch, r, world)[1] - pair_range(batch, r, world)[0] for r in range(world))
        recv = [torch.empty((width, 6, 10), dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
        parts = gather_disparity(local, batch, recv=recv, concat=False)
        if rank == 0:
            parts = torch.cat(parts, 0)
        if rank == 0:
            exp = torch.stack([(torch.arange(60, dtype=torch.int32).reshape(6, 10) + 7 * i) % 256
                               for i in range(batch)]).to(torch.uint8)
            q.put(("ok", bool(torch.equal(out, exp)) and bool(torch.equal(pend, exp))
                   and bool(torch.equal(parts, exp))))
        else:
            q.put(("none", out is None and pend is None and parts is None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch", [2, 5])
def test_gather_world2_gloo(batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, batch, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v for _, v in res), res

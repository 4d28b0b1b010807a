"""Multi-GPU data parallelism over independent stereo pairs.

Two forms: a batch of pairs, one (or a few) per GPU (weak scaling, configs D / E: pair_range +
gather_disparity), and one frame split into row bands with halos (strong scaling of config C:
band_range + match_band + gather_bands).

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


# ---- single-frame band sharding (SURVEY.md §8(e), config C at N GPUs) ----

def band_range(H: int, rank: int, world: int, window: int) -> tuple[int, int, int, int]:
    """Rows of one frame for `rank`: output rows [y0, y1) and the input rows [i0, i1) it reads.

    The input band adds r = (window - 1) / 2 halo rows on each side, cut at the image: the block
    matcher's row clamp then only ever applies at the true image borders, so a band's output rows
    are bit-identical to the same rows of the full-frame result (tests/test_sharding.py).
    """
    if window < 1 or window % 2 == 0:
        raise ValueError("window must be odd and positive")
    y0, y1 = pair_range(H, rank, world)
    r = (window - 1) // 2
    return y0, y1, max(0, y0 - r), min(H, y1 + r)


def match_band(matcher, left, right, rank: int, world: int, out=None):
    """Disparity of rank's output rows of one (H, W) frame: the matcher runs on the halo'd input
    band (a row view, no copy) and the band's own rows are returned (a view of `out` if given)."""
    H = left.shape[0]
    y0, y1, i0, i1 = band_range(H, rank, world, matcher.window)
    full = matcher.compute(left[i0:i1], right[i0:i1], out_disp=out)
    return full[y0 - i0:y1 - i0]


def gather_bands(local, H: int, dst: int = 0, group=None, recv: list | None = None):
    """Collect every rank's (y1 - y0, W) u8 band into the (H, W) frame on `dst` (one gather; ranks
    pad to the largest band).  Returns the frame on dst, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    y0, y1 = pair_range(H, rank, world)
    if local.shape[0] != y1 - y0:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, band is {y1 - y0}")
    width = max(pair_range(H, r, world)[1] - pair_range(H, r, world)[0] for r in range(world))
    send = local
    if local.shape[0] < width:
        send = torch.cat([local, torch.zeros((width - local.shape[0],) + tuple(local.shape[1:]),
                                             dtype=local.dtype, device=local.device)], 0)
    bufs = None
    if rank == dst:
        bufs = recv if recv is not None else [torch.empty_like(send) for _ in range(world)]
    dist.gather(send.contiguous(), bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([bufs[r][:pair_range(H, r, world)[1] - pair_range(H, r, world)[0]] for r in range(world)], 0)


# ---- one process, several GPUs: the C-ABI engine (include/usv.h usv_sharded_*) ----

class ShardedMatcher:
    """usv_sharded_engine through ctypes: one process drives `devices` (HIP ordinals), one stream and
    RCCL communicator per GPU; pairs shard like pair_range and one ncclGather brings the u8 maps to
    devices[0] (csrc/usv_sharded.hip).  This is the entry the reference's single C++ process would use;
    bench.py's one-process-per-GPU torch.distributed path is the other form of the same split."""

    def __init__(self, devices, max_pairs: int, W: int, H: int, D: int, w: int, metric: str = "sad"):
        import ctypes

        from . import _lib
        self._ct, self._lib_mod = ctypes, _lib
        self.lib = _lib.load()
        self.devices = list(devices)
        self.W, self.H, self.max_pairs = W, H, max_pairs
        devs = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        _lib.check("usv_sharded_create", self.lib.usv_sharded_create(
            devs, len(self.devices), max_pairs, W, H, D, w, {"sad": 0, "ssd": 1}[metric], ctypes.byref(h)))
        self.handle = h

    def close(self):
        if self.handle:
            self._lib_mod.check("usv_sharded_destroy", self.lib.usv_sharded_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def input_buffers(self, k: int):
        """Device pointers (L, R) of GPU k's dense shard inputs."""
        ct = self._ct
        L, R = ct.c_void_p(), ct.c_void_p()
        self._lib_mod.check("usv_sharded_input_buffers",
                            self.lib.usv_sharded_input_buffers(self.handle, k, ct.byref(L), ct.byref(R)))
        return L.value, R.value

    def outputs(self):
        """Device pointers (gathered u8 disparity on devices[0], distance maps or None)."""
        ct = self._ct
        d, x = ct.c_void_p(), ct.c_void_p()
        self._lib_mod.check("usv_sharded_outputs", self.lib.usv_sharded_outputs(self.handle, ct.byref(d),
                                                                                 ct.byref(x)))
        return d.value, x.value

    def run(self, L=None, R=None, batch: int | None = None, with_distance: bool = False, lut=None,
            want_host: bool = True):
        """Host numpy batches (B, H, W) u8 -> (disp (B, H, W) u8, dist (B, H, W) f64 or None), or with
        L = R = None the frames already in input_buffers (then `batch` is required)."""
        import numpy as np
        ct = self._ct
        if L is not None:
            L = np.ascontiguousarray(L)
            R = np.ascontiguousarray(R)
            if L.shape != R.shape or L.ndim != 3 or L.shape[1:] != (self.H, self.W) or L.dtype != np.uint8:
                raise ValueError("L, R must be (B, H, W) uint8 batches of the engine's geometry")
            batch = L.shape[0]
        if batch is None:
            raise ValueError("batch is required for resident inputs")
        disp = np.empty((batch, self.H, self.W), np.uint8) if want_host else None
        dist = np.empty((batch, self.H, self.W), np.float64) if (with_distance and want_host) else None
        if with_distance and lut is None:
            from .engine import distance_lut_cm
            lut = distance_lut_cm()
        lut_arr = np.ascontiguousarray(lut, dtype=np.float64) if lut is not None else None
        vp = lambda a: a.ctypes.data_as(ct.c_void_p) if a is not None else None  # noqa: E731
        self._lib_mod.check("usv_batch_sharded", self.lib.usv_batch_sharded(
            self.handle, vp(L), vp(R), batch, self.H * self.W, self.W, vp(disp), vp(dist), vp(lut_arr),
            int(bool(with_distance))))
        return disp, dist

    def submit(self, L, R, with_distance: bool = False, lut=None):
        """Enqueue a host batch on the engine's next buffer slot (usv_batch_sharded_submit) and return a
        handle for wait(); two batches can be in flight."""
        import numpy as np
        ct = self._ct
        L = np.ascontiguousarray(L)
        R = np.ascontiguousarray(R)
        if L.shape != R.shape or L.ndim != 3 or L.shape[1:] != (self.H, self.W) or L.dtype != np.uint8:
            raise ValueError("L, R must be (B, H, W) uint8 batches of the engine's geometry")
        batch = L.shape[0]
        disp = np.empty((batch, self.H, self.W), np.uint8)
        dist = np.empty((batch, self.H, self.W), np.float64) if with_distance else None
        if with_distance and lut is None:
            from .engine import distance_lut_cm
            lut = distance_lut_cm()
        lut_arr = np.ascontiguousarray(lut, dtype=np.float64) if lut is not None else None
        vp = lambda a: a.ctypes.data_as(ct.c_void_p) if a is not None else None  # noqa: E731
        t = ct.c_longlong()
        self._lib_mod.check("usv_batch_sharded_submit", self.lib.usv_batch_sharded_submit(
            self.handle, vp(L), vp(R), batch, self.H * self.W, self.W, vp(disp), vp(dist), vp(lut_arr),
            int(bool(with_distance)), ct.byref(t)))
        # the host outputs (and the table) must outlive the batch: keep them with the ticket
        return {"ticket": t.value, "disp": disp, "dist": dist, "keep": (L, R, lut_arr)}

    def wait(self, h):
        """Complete a submitted batch: (disp, dist or None) in batch order."""
        self._lib_mod.check("usv_batch_sharded_wait", self.lib.usv_batch_sharded_wait(self.handle, h["ticket"]))
        return h["disp"], h["dist"]

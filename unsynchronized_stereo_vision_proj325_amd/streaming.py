"""Streaming HOST frames through the matcher (usv_frame_stream_*, include/usv.h).

The reference's caller hands over host frames, one pair per camera-thread
iteration (P/Main.cpp:876-921, 1238-1242).  ``FrameStream`` keeps ``depth``
pairs in flight so that the PCIe copies of neighbouring frames overlap the
match: frame k+1's H2D, frame k's kernel and frame k-1's D2H run at once.
Outputs are u8 disparity maps in pinned host memory; per-pixel distances are
expanded on the host from the 256-entry table (``expand_distance``) only when
asked, or computed on the device with ``device_distance=True``.

    fs = FrameStream(W, H, D=128, w=11)
    L, R = fs.next_inputs()          # pinned numpy views: fill them (zero-copy submit)
    L[:] = ...; R[:] = ...
    t = fs.submit(L, R)
    disp = fs.wait(t)                # numpy view of pinned memory, valid until release
    fs.release(t)
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np

from . import _lib
from .engine import distance_lut_cm

_METRICS = {"sad": _lib.METRIC_SAD, "ssd": _lib.METRIC_SSD}


class _PinnedView:
    """Array interface over a FrameStream's pinned memory that holds a reference to the stream: a numpy
    view's base is this object, so while any view (or a slice of one) is alive the stream -- and the
    pinned allocation behind it -- cannot be collected, and an explicit close() defers the free until
    the last view is gone (FrameStream._nviews)."""

    def __init__(self, owner, ptr: int, shape, dtype):
        self._owner = owner
        self.__array_interface__ = {"data": (ptr, False), "shape": tuple(shape), "typestr": np.dtype(dtype).str,
                                    "version": 3}


def _view(owner, ptr: int, shape, dtype) -> np.ndarray:
    holder = _PinnedView(owner, ptr, shape, dtype)
    owner._nviews += 1
    weakref.finalize(holder, owner._view_gone)
    return np.asarray(holder)


class FrameStream:
    """``depth`` frames in flight on the current HIP device (usv_frame_stream_create)."""

    def __init__(self, W: int, H: int, D: int = 128, w: int = 11, metric: str = "sad", depth: int = 3,
                 device_distance: bool = False):
        self._lib = _lib.load()
        self._nviews = 0  # live _PinnedView holders (numpy views of the pinned staging)
        self._closing = False
        self.W, self.H, self.D, self.w = W, H, D, w
        self.device_distance = device_distance
        h = ctypes.c_void_p()
        flags = _lib.STREAM_DEVICE_DIST if device_distance else 0
        _lib.check("usv_frame_stream_create",
                   self._lib.usv_frame_stream_create(W, H, D, w, _METRICS[metric], depth, flags, ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        """Destroy the stream (its pinned host memory included).  While numpy views returned by
        next_inputs() / wait() are still alive the free is deferred until the last one is collected,
        so a view can never point at released memory; the stream takes no new submits meanwhile."""
        self._closing = True
        if self._h and self._nviews == 0:
            self._destroy()

    def _view_gone(self) -> None:  # a view's holder was collected
        self._nviews -= 1
        if self._closing and self._nviews == 0 and self._h:
            self._destroy()

    def _destroy(self) -> None:
        h, self._h = self._h, None
        _lib.check("usv_frame_stream_destroy", self._lib.usv_frame_stream_destroy(h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _require_open(self) -> None:
        if self._closing or not self._h:
            raise RuntimeError("FrameStream is closed")

    def next_inputs(self) -> tuple[np.ndarray, np.ndarray]:
        """Pinned (H, W) u8 staging of the next submit's slot (write the frames there)."""
        self._require_open()
        lp, rp = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check("usv_frame_stream_next_inputs",
                   self._lib.usv_frame_stream_next_inputs(self._h, ctypes.byref(lp), ctypes.byref(rp)))
        return _view(self, lp.value, (self.H, self.W), np.uint8), _view(self, rp.value, (self.H, self.W), np.uint8)

    def submit(self, L: np.ndarray, R: np.ndarray) -> int:
        """Enqueue one host pair ((H, W) u8, unit column stride); returns the frame's ticket."""
        self._require_open()
        for a, n in ((L, "L"), (R, "R")):
            if not isinstance(a, np.ndarray) or a.dtype != np.uint8 or a.shape != (self.H, self.W) or \
                    a.strides[1] != 1:
                raise ValueError(f"{n} must be a ({self.H}, {self.W}) uint8 array with unit column stride")
        if L.strides != R.strides:
            raise ValueError("L and R must share one row pitch")
        t = ctypes.c_longlong()
        _lib.check("usv_frame_stream_submit",
                   self._lib.usv_frame_stream_submit(self._h, L.ctypes.data, R.ctypes.data, L.strides[0],
                                                     ctypes.byref(t)))
        return t.value

    def wait(self, ticket: int):
        """Block until frame `ticket` is done: its (H, W) u8 disparity (pinned memory, valid until
        release), plus the f64 cm distance map when the stream computes it on the device."""
        self._require_open()
        dp, xp = ctypes.c_void_p(), ctypes.c_void_p()
        _lib.check("usv_frame_stream_wait",
                   self._lib.usv_frame_stream_wait(self._h, ticket, ctypes.byref(dp),
                                                   ctypes.byref(xp) if self.device_distance else None))
        disp = _view(self, dp.value, (self.H, self.W), np.uint8)
        if self.device_distance:
            return disp, _view(self, xp.value, (self.H, self.W), np.float64)
        return disp

    def release(self, ticket: int) -> None:
        self._require_open()
        _lib.check("usv_frame_stream_release", self._lib.usv_frame_stream_release(self._h, ticket))


def expand_distance(disp: np.ndarray, lut: np.ndarray | None = None, threads: int = 1,
                    out: np.ndarray | None = None) -> np.ndarray:
    """Host distance map lut[disp] (usv_distance_expand_host); default table: the reference's
    moving-object law in cm (P/DistanceCalculator.cpp:84)."""
    lib = _lib.load()
    if lut is None:
        lut = distance_lut_cm()
    lut = np.ascontiguousarray(lut, dtype=np.float64)
    if lut.shape != (256,) or disp.dtype != np.uint8 or disp.ndim != 2 or disp.strides[1] != 1:
        raise ValueError("disp must be (H, W) uint8 with unit column stride and lut 256 doubles")
    H, W = disp.shape
    if out is None:
        out = np.empty((H, W), dtype=np.float64)
    _lib.check("usv_distance_expand_host",
               lib.usv_distance_expand_host(disp.ctypes.data, W, H, disp.strides[0], lut.ctypes.data,
                                            out.ctypes.data, out.strides[0] // 8, threads))
    return out

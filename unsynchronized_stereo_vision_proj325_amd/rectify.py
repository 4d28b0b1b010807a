"""Stereo rectification on the GPU.

The reference rectifies every frame of each camera with
``initUndistortRectifyMap(K, dist, R, P, size, CV_16SC2)`` + ``remap(INTER_LINEAR,
BORDER_CONSTANT)`` (P/Main.cpp:351-359), rebuilding the map each time because
the calibration struct is passed by value.  ``Rectifier`` builds the map once on
the device (usv_rectify_map) and remaps each frame with one HBM-bound gather
(usv_remap_linear_u8); ``rectify_pair`` does both cameras in one launch.  When the
source is at most 2046 x 2046 the map is also packed into one u32 per pixel
(usv_remap_pack_map: 4 B instead of 6, bit-identical results) and the frames go
through the packed form.
Calibration matrices are the ones ``calibration.load_calibration`` reads.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .engine import _stream


def rectify_params(K, dist, R, P) -> np.ndarray:
    """Host: the 25 doubles initUndistortRectifyMap derives (include/usv.h usv_rectify_params)."""
    lib = _lib.load()
    K = np.ascontiguousarray(K, dtype=np.float64).reshape(3, 3)
    P = np.ascontiguousarray(P, dtype=np.float64)
    if P.shape not in ((3, 3), (3, 4)):
        raise ValueError("P must be 3x3 or 3x4")
    d = np.ascontiguousarray(np.zeros(0) if dist is None else dist, dtype=np.float64).ravel()
    Rm = None if R is None else np.ascontiguousarray(R, dtype=np.float64).reshape(3, 3)
    out = np.zeros(25, dtype=np.float64)
    _lib.check("usv_rectify_params",
               lib.usv_rectify_params(K.ctypes.data, d.ctypes.data if d.size else None, int(d.size),
                                      Rm.ctypes.data if Rm is not None else None, P.ctypes.data,
                                      int(P.shape[1]), out.ctypes.data))
    return out


def _check_u8(t: torch.Tensor, name: str) -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.uint8:
        raise ValueError(f"{name} must be a uint8 CUDA (HIP) tensor; there is no CPU path")
    if t.dim() not in (2, 3) or t.stride(-1) != 1 or (t.dim() == 3 and t.stride(-2) != t.shape[-1]):
        raise ValueError(f"{name} must be (H, W) or (H, W, C) with interleaved channels")


class Rectifier:
    """One camera's rectification: map built once on `device`, applied per frame."""

    PACK_MAX_SRC = 2046  # include/usv.h usv_remap_pack_map

    TILE_W, TILE_H = 64, 16  # include/usv.h usv_remap_tile_boxes

    def __init__(self, K, dist, R, P, size: tuple[int, int], device=None, stream=None,
                 src_size: tuple[int, int] | None = None, packed: bool = True, tiled: bool = False):
        """size: output (W, H); src_size: the frames' (W, H) (default: size, as initUndistortRectifyMap's
        callers use it, P/Main.cpp:352); packed: also build the packed map when the source allows; tiled:
        remap packed frames through the LDS-tiled kernel (source boxes per 64 x 16 tile, built once per
        channel count on first use; bit-identical to the direct packed remap).  Off by default: measured
        slower than the direct packed remap (12.7 vs 12.0-12.4 us for the 1080p BGR pair)."""
        self.tiled = tiled
        self._boxes = {}
        self.W, self.H = int(size[0]), int(size[1])
        self.sW, self.sH = (self.W, self.H) if src_size is None else (int(src_size[0]), int(src_size[1]))
        self.params = rectify_params(K, dist, R, P)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.map1 = torch.empty((self.H, self.W, 2), dtype=torch.int16, device=dev)
        self.map2 = torch.empty((self.H, self.W), dtype=torch.int16, device=dev)  # bit pattern of uint16
        lib = _lib.load()
        p = np.ascontiguousarray(self.params)
        with torch.cuda.device(dev):
            _lib.check("usv_rectify_map", lib.usv_rectify_map(p.ctypes.data, self.W, self.H, self.map1.data_ptr(),
                                                              self.map2.data_ptr(), _stream(stream)))
        self.pmap = None
        if packed and self.sW <= self.PACK_MAX_SRC and self.sH <= self.PACK_MAX_SRC:
            self.pmap = torch.empty((self.H, self.W), dtype=torch.int32, device=dev)  # bit pattern of uint32
            with torch.cuda.device(dev):
                _lib.check("usv_remap_pack_map", lib.usv_remap_pack_map(
                    self.map1.data_ptr(), self.map2.data_ptr(), self.W, self.H, self.sW, self.sH,
                    self.pmap.data_ptr(), _stream(stream)))

    def boxes(self, cn: int, stream=None) -> torch.Tensor:
        """The packed map's per-tile source boxes for cn-channel frames (usv_remap_tile_boxes), cached."""
        if cn not in self._boxes:
            tiles = ((self.W + self.TILE_W - 1) // self.TILE_W) * ((self.H + self.TILE_H - 1) // self.TILE_H)
            b = torch.empty((tiles, 2), dtype=torch.int32, device=self.pmap.device)
            with torch.cuda.device(self.pmap.device):
                _lib.check("usv_remap_tile_boxes", _lib.load().usv_remap_tile_boxes(
                    self.pmap.data_ptr(), self.W, self.H, self.sW, self.sH, cn, b.data_ptr(), _stream(stream)))
            self._boxes[cn] = b
        return self._boxes[cn]

    def packed_for(self, src: torch.Tensor) -> bool:
        """True when frames of src's size go through the packed map."""
        return self.pmap is not None and (src.shape[1], src.shape[0]) == (self.sW, self.sH)

    def maps_numpy(self):
        """(map1 int16 (H, W, 2), map2 uint16 (H, W)) on the host, OpenCV's CV_16SC2 / CV_16UC1 layout."""
        return self.map1.cpu().numpy(), self.map2.cpu().numpy().view(np.uint16)

    def __call__(self, src: torch.Tensor, out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
        _check_u8(src, "src")
        cn = 1 if src.dim() == 2 else src.shape[2]
        if out is None:
            out = torch.empty((self.H, self.W) if cn == 1 else (self.H, self.W, cn), dtype=torch.uint8,
                              device=src.device)
        _check_u8(out, "out")
        lib = _lib.load()
        if self.packed_for(src) and self.tiled:
            boxes = self.boxes(cn, stream)
            with torch.cuda.device(src.device):
                _lib.check("usv_remap_packed_tiled_u8", lib.usv_remap_packed_tiled_u8(
                    src.data_ptr(), src.shape[1], src.shape[0], src.stride(0), cn, self.pmap.data_ptr(),
                    boxes.data_ptr(), self.W, self.H, out.data_ptr(), out.stride(0), _stream(stream)))
            return out
        if self.packed_for(src):
            with torch.cuda.device(src.device):
                _lib.check("usv_remap_packed_u8", lib.usv_remap_packed_u8(
                    src.data_ptr(), src.shape[1], src.shape[0], src.stride(0), cn, self.pmap.data_ptr(), self.W,
                    self.H, out.data_ptr(), out.stride(0), _stream(stream)))
            return out
        with torch.cuda.device(src.device):
            _lib.check("usv_remap_linear_u8", lib.usv_remap_linear_u8(
                src.data_ptr(), src.shape[1], src.shape[0], src.stride(0), cn, self.map1.data_ptr(),
                self.map2.data_ptr(), self.W, self.H, out.data_ptr(), out.stride(0), _stream(stream)))
        return out


def rectify_pair(left: Rectifier, right: Rectifier, src_l: torch.Tensor, src_r: torch.Tensor,
                 out_l: torch.Tensor | None = None, out_r: torch.Tensor | None = None, stream=None):
    """Both cameras in one launch (usv_rectify_pair_u8)."""
    _check_u8(src_l, "src_l")
    _check_u8(src_r, "src_r")
    if src_l.shape != src_r.shape or src_l.stride() != src_r.stride():
        raise ValueError("the two sources must share shape and strides")
    if (left.W, left.H) != (right.W, right.H):
        raise ValueError("the two rectifiers must share the output size")
    cn = 1 if src_l.dim() == 2 else src_l.shape[2]
    shape = (left.H, left.W) if cn == 1 else (left.H, left.W, cn)
    out_l = torch.empty(shape, dtype=torch.uint8, device=src_l.device) if out_l is None else out_l
    out_r = torch.empty(shape, dtype=torch.uint8, device=src_l.device) if out_r is None else out_r
    if out_l.stride() != out_r.stride():
        raise ValueError("the two outputs must share strides")
    lib = _lib.load()
    if left.packed_for(src_l) and right.packed_for(src_r) and left.tiled and right.tiled:
        bl, br = left.boxes(cn, stream), right.boxes(cn, stream)
        with torch.cuda.device(src_l.device):
            _lib.check("usv_rectify_pair_packed_tiled_u8", lib.usv_rectify_pair_packed_tiled_u8(
                src_l.data_ptr(), src_r.data_ptr(), src_l.shape[1], src_l.shape[0], src_l.stride(0), cn,
                left.pmap.data_ptr(), right.pmap.data_ptr(), bl.data_ptr(), br.data_ptr(), left.W, left.H,
                out_l.data_ptr(), out_r.data_ptr(), out_l.stride(0), _stream(stream)))
        return out_l, out_r
    if left.packed_for(src_l) and right.packed_for(src_r):
        with torch.cuda.device(src_l.device):
            _lib.check("usv_rectify_pair_packed_u8", lib.usv_rectify_pair_packed_u8(
                src_l.data_ptr(), src_r.data_ptr(), src_l.shape[1], src_l.shape[0], src_l.stride(0), cn,
                left.pmap.data_ptr(), right.pmap.data_ptr(), left.W, left.H, out_l.data_ptr(), out_r.data_ptr(),
                out_l.stride(0), _stream(stream)))
        return out_l, out_r
    with torch.cuda.device(src_l.device):
        _lib.check("usv_rectify_pair_u8", lib.usv_rectify_pair_u8(
            src_l.data_ptr(), src_r.data_ptr(), src_l.shape[1], src_l.shape[0], src_l.stride(0), cn,
            left.map1.data_ptr(), left.map2.data_ptr(), right.map1.data_ptr(), right.map2.data_ptr(),
            left.W, left.H, out_l.data_ptr(), out_r.data_ptr(), out_l.stride(0), _stream(stream)))
    return out_l, out_r


def synthetic_calibration(W: int, H: int, seed: int = 0, distortion: bool = True):
    """A plausible stereo calibration for tests and the bench (there is no calibration file in the
    reference tree): K, dist (5 or 8 terms), R (small rotation), P (3x4), for each camera."""
    rng = np.random.default_rng(seed)
    cams = []
    for side in range(2):
        f = W * (0.9 + 0.1 * rng.random())
        K = np.array([[f, 0, W / 2 + rng.uniform(-8, 8)], [0, f * (1 + rng.uniform(-0.01, 0.01)),
                                                             H / 2 + rng.uniform(-8, 8)], [0, 0, 1]])
        dist = np.array([rng.uniform(-0.3, 0.1), rng.uniform(-0.1, 0.1), rng.uniform(-1e-3, 1e-3),
                         rng.uniform(-1e-3, 1e-3), rng.uniform(-0.05, 0.05)]) if distortion else np.zeros(5)
        a, b, c = rng.uniform(-0.02, 0.02, size=3)
        Rx = np.array([[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]])
        Ry = np.array([[np.cos(b), 0, np.sin(b)], [0, 1, 0], [-np.sin(b), 0, np.cos(b)]])
        Rz = np.array([[np.cos(c), -np.sin(c), 0], [np.sin(c), np.cos(c), 0], [0, 0, 1]])
        R = Rz @ Ry @ Rx
        fn = f * 0.95
        P = np.array([[fn, 0, W / 2, -fn * 0.06 * side], [0, fn, H / 2, 0], [0, 0, 1, 0]])
        cams.append((K, dist, R, P))
    return cams

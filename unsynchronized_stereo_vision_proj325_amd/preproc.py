"""Per-frame colour chain and masks on the GPU.

Mirrors what the reference does to every rectified frame (P/Main.cpp:915-921
and the search helpers it calls), with the reference's function names where it
has them:

  ``frame_prep``        cvtColor BGR2HSV -> LightingCorrection (split /
                        equalizeHist(V) / merge / HSV2BGR) -> cvtColor BGR2GRAY
                        (P/Main.cpp:919-921, 365-371); returns (hsv', bgr', gray)
  ``ABSDiffSearch``     absdiff with the previous gray frame, threshold 40,
                        MorphilogicalFilter (P/Main.cpp:299-312, 289-292)
  ``ColourSearch``      two inRange + addWeighted + MorphilogicalFilter
                        (P/Main.cpp:318-327)

All compute is in libusv.so (csrc/usv_preproc.hip); inputs must be uint8 GPU
tensors.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .engine import _stream


def _u8(t: torch.Tensor, name: str, channels: int) -> None:
    if not isinstance(t, torch.Tensor) or not t.is_cuda or t.dtype != torch.uint8:
        raise ValueError(f"{name} must be a uint8 CUDA (HIP) tensor; there is no CPU path")
    want = 2 if channels == 1 else 3
    if t.dim() != want or (channels > 1 and t.shape[2] != channels) or t.stride(-1) != 1:
        raise ValueError(f"{name} must be {'(H, W)' if channels == 1 else f'(H, W, {channels})'} contiguous rows")
    if channels > 1 and t.stride(1) != channels:
        raise ValueError(f"{name} must hold interleaved channels")


class FramePrep:
    """Reusable device workspace (two alternating 256-bin histograms; include/usv.h) for frame_prep on
    one device.  One FramePrep per stream in flight."""

    WORK_WORDS = 2 * 8 * 256  # USV_FRAME_PREP_WORK_BYTES / 4

    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.work = torch.zeros(self.WORK_WORDS, dtype=torch.int32, device=dev)
        self.parity = 0

    @property
    def hist(self) -> torch.Tensor:
        """The last frame's 256-bin histogram of V (equalizeHist's input)."""
        p = 1 - self.parity
        return self.work[2048 * p:2048 * (p + 1)].view(8, 256).sum(0)

    def __call__(self, bgr: torch.Tensor, hsv: torch.Tensor | None = None, bgr_out: torch.Tensor | None = None,
                 gray: torch.Tensor | None = None, stream=None):
        _u8(bgr, "bgr", 3)
        H, W = bgr.shape[:2]
        hsv = torch.empty((H, W, 3), dtype=torch.uint8, device=bgr.device) if hsv is None else hsv
        bgr_out = torch.empty((H, W, 3), dtype=torch.uint8, device=bgr.device) if bgr_out is None else bgr_out
        gray = torch.empty((H, W), dtype=torch.uint8, device=bgr.device) if gray is None else gray
        _u8(hsv, "hsv", 3)
        _u8(bgr_out, "bgr_out", 3)
        _u8(gray, "gray", 1)
        lib = _lib.load()
        with torch.cuda.device(bgr.device):
            _lib.check("usv_frame_prep_u8", lib.usv_frame_prep_u8(
                bgr.data_ptr(), W, H, bgr.stride(0), hsv.data_ptr(), hsv.stride(0), bgr_out.data_ptr(),
                bgr_out.stride(0), gray.data_ptr(), gray.stride(0), self.work.data_ptr(), self.parity,
                _stream(stream)))
        self.parity ^= 1
        return hsv, bgr_out, gray


def frame_prep(bgr: torch.Tensor, stream=None):
    """(hsv', bgr', gray) of one rectified BGR frame; see FramePrep."""
    return FramePrep(bgr.device)(bgr, stream=stream)


class FramePrepPair:
    """Both cameras' frame preparation in two launches (usv_frame_prep_pair_u8), or the whole per-frame
    stage including rectification (usv_rectify_prep_pair_u8, rectify_prep).  Owns one workspace per
    camera (2 x USV_FRAME_PREP_WORK_BYTES) and alternates its parity per call."""

    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.work = torch.zeros(2 * FramePrep.WORK_WORDS, dtype=torch.int32, device=dev)
        self.parity = 0

    def hist(self, camera: int) -> torch.Tensor:
        """The last frame's 256-bin histogram of V of camera 0 (L) or 1 (R)."""
        p = 1 - self.parity
        base = camera * FramePrep.WORK_WORDS
        return self.work[base + 2048 * p:base + 2048 * (p + 1)].view(8, 256).sum(0)

    @staticmethod
    def _outs(ref: torch.Tensor, H: int, W: int, outs):
        if outs is None:
            outs = [torch.empty((H, W, 3), dtype=torch.uint8, device=ref.device) for _ in range(4)] + \
                   [torch.empty((H, W), dtype=torch.uint8, device=ref.device) for _ in range(2)]
        hl, hr, bl, br, gl, gr = outs
        for t, n in ((hl, "hsvL"), (hr, "hsvR"), (bl, "bgrL"), (br, "bgrR")):
            _u8(t, n, 3)
        _u8(gl, "grayL", 1)
        _u8(gr, "grayR", 1)
        if hl.stride() != hr.stride() or bl.stride() != br.stride() or gl.stride() != gr.stride():
            raise ValueError("the two cameras' outputs must share their row pitches")
        return outs

    def __call__(self, bgr_l: torch.Tensor, bgr_r: torch.Tensor, outs=None, stream=None):
        """((hsv'_L, hsv'_R), (bgr'_L, bgr'_R), (gray_L, gray_R)) of a rectified BGR pair."""
        _u8(bgr_l, "bgr_l", 3)
        _u8(bgr_r, "bgr_r", 3)
        if bgr_l.shape != bgr_r.shape or bgr_l.stride() != bgr_r.stride():
            raise ValueError("the two frames must share shape and strides")
        H, W = bgr_l.shape[:2]
        hl, hr, bl, br, gl, gr = self._outs(bgr_l, H, W, outs)
        lib = _lib.load()
        with torch.cuda.device(bgr_l.device):
            _lib.check("usv_frame_prep_pair_u8", lib.usv_frame_prep_pair_u8(
                bgr_l.data_ptr(), bgr_r.data_ptr(), W, H, bgr_l.stride(0), hl.data_ptr(), hr.data_ptr(),
                hl.stride(0), bl.data_ptr(), br.data_ptr(), bl.stride(0), gl.data_ptr(), gr.data_ptr(),
                gl.stride(0), self.work.data_ptr(), self.parity, _stream(stream)))
        self.parity ^= 1
        return (hl, hr), (bl, br), (gl, gr)

    def rectify_prep(self, left, right, src_l: torch.Tensor, src_r: torch.Tensor, outs=None, stream=None):
        """The same outputs from the RAW BGR frames and the two cameras' Rectifier maps, in two launches
        (rectification fused into the HSV + histogram pass; no rectified-BGR intermediate)."""
        _u8(src_l, "src_l", 3)
        _u8(src_r, "src_r", 3)
        if src_l.shape != src_r.shape or src_l.stride() != src_r.stride():
            raise ValueError("the two frames must share shape and strides")
        sH, sW = src_l.shape[:2]
        W, H = left.W, left.H
        if (right.W, right.H) != (W, H):
            raise ValueError("the two rectifiers must share the output size")
        hl, hr, bl, br, gl, gr = self._outs(src_l, H, W, outs)
        lib = _lib.load()
        if left.packed_for(src_l) and right.packed_for(src_r):
            with torch.cuda.device(src_l.device):
                _lib.check("usv_rectify_prep_pair_packed_u8", lib.usv_rectify_prep_pair_packed_u8(
                    src_l.data_ptr(), src_r.data_ptr(), sW, sH, src_l.stride(0), left.pmap.data_ptr(),
                    right.pmap.data_ptr(), W, H, hl.data_ptr(), hr.data_ptr(), hl.stride(0), bl.data_ptr(),
                    br.data_ptr(), bl.stride(0), gl.data_ptr(), gr.data_ptr(), gl.stride(0), self.work.data_ptr(),
                    self.parity, _stream(stream)))
            self.parity ^= 1
            return (hl, hr), (bl, br), (gl, gr)
        with torch.cuda.device(src_l.device):
            _lib.check("usv_rectify_prep_pair_u8", lib.usv_rectify_prep_pair_u8(
                src_l.data_ptr(), src_r.data_ptr(), sW, sH, src_l.stride(0), left.map1.data_ptr(),
                left.map2.data_ptr(), right.map1.data_ptr(), right.map2.data_ptr(), W, H, hl.data_ptr(),
                hr.data_ptr(), hl.stride(0), bl.data_ptr(), br.data_ptr(), bl.stride(0), gl.data_ptr(),
                gr.data_ptr(), gl.stride(0), self.work.data_ptr(), self.parity, _stream(stream)))
        self.parity ^= 1
        return (hl, hr), (bl, br), (gl, gr)


def ABSDiffSearch(gray: torch.Tensor, prev: torch.Tensor | None, thresh: int = 40,
                  out: torch.Tensor | None = None, stream=None):
    """Motion mask of P/Main.cpp:299-312.  Returns (mask, next_prev): as in the
    reference, an empty previous frame is replaced by the current one (first
    call -> all-zero mask) and the current gray frame becomes the next prev."""
    _u8(gray, "gray", 1)
    if prev is None:
        prev = gray
    _u8(prev, "prev", 1)
    if prev.shape != gray.shape or prev.stride() != gray.stride():
        raise ValueError("prev must match gray's shape and strides")
    H, W = gray.shape
    out = torch.empty((H, W), dtype=torch.uint8, device=gray.device) if out is None else out
    _u8(out, "out", 1)
    lib = _lib.load()
    with torch.cuda.device(gray.device):
        _lib.check("usv_motion_mask_u8", lib.usv_motion_mask_u8(
            gray.data_ptr(), prev.data_ptr(), W, H, gray.stride(0), int(thresh), out.data_ptr(), out.stride(0),
            _stream(stream)))
    return out, gray


@dataclass
class ColourSearchParameters:
    """P/Main.cpp:159-165 (slider values): hue range 1 and 2, shared S and V ranges."""
    iLowHue: int = 0
    iLowSaturation: int = 0
    iLowValue: int = 0
    iHighHue: int = 179
    iHighSaturation: int = 255
    iHighValue: int = 255
    iLowHue2: int = 0
    iHighHue2: int = 0


def ColourSearch(hsv: torch.Tensor, p: ColourSearchParameters, out: torch.Tensor | None = None, stream=None):
    """Colour mask of P/Main.cpp:318-327 on an HSV frame."""
    _u8(hsv, "hsv", 3)
    H, W = hsv.shape[:2]
    lo1 = np.array([p.iLowHue, p.iLowSaturation, p.iLowValue], dtype=np.int32)
    hi1 = np.array([p.iHighHue, p.iHighSaturation, p.iHighValue], dtype=np.int32)
    lo2 = np.array([p.iLowHue2, p.iLowSaturation, p.iLowValue], dtype=np.int32)
    hi2 = np.array([p.iHighHue2, p.iHighSaturation, p.iHighValue], dtype=np.int32)
    out = torch.empty((H, W), dtype=torch.uint8, device=hsv.device) if out is None else out
    _u8(out, "out", 1)
    lib = _lib.load()
    with torch.cuda.device(hsv.device):
        _lib.check("usv_colour_mask_u8", lib.usv_colour_mask_u8(
            hsv.data_ptr(), W, H, hsv.stride(0), lo1.ctypes.data, hi1.ctypes.data, lo2.ctypes.data,
            hi2.ctypes.data, out.data_ptr(), out.stride(0), _stream(stream)))
    return out

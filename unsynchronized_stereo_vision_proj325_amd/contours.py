"""Batched contour matcher on the GPU.

``GenerateMatchingListGPU`` returns what ``GenerateMatchingList``
(P/Main.cpp:403-426, host restatement in csrc/host/matching.cpp) returns --
(i, j, v) for every pair with v < 0.75, i-major then j-minor -- but computes
each contour's Hu-moment I1 terms and area once on the device
(``usv_contour_descriptors``) and all N×M scores in one launch
(``usv_contour_pair_scores``), instead of the reference's per-pair
recomputation.  ``ContourMatcherGPU`` (usv_generate_matching_list_gpu) does the
whole call on the device: one copy in, the descriptor launches, a selection
launch that keeps v < 0.75 and compacts each row in order, one copy out.

OpenCV 3.0 is absent, so parity with OpenCV itself is UNPINNED; the device
scores equal the host restatement's to the ulp (log10 is the only libm call,
tests/test_gpu_contours.py).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .engine import _stream
from .host import _flatten

DESC = 8  # doubles per contour: 7 I1 terms + |area|


def contour_descriptors(contours, device="cuda", stream=None) -> torch.Tensor:
    """(n, 8) float64 device tensor of per-contour I1 terms (NaN = skipped invariant) and unoriented area."""
    lib = _lib.load()
    pts, off = _flatten(contours)
    n = len(contours)
    d_pts = torch.from_numpy(pts).to(device)
    d_off = torch.from_numpy(off).to(device)
    desc = torch.empty((max(n, 1), DESC), dtype=torch.float64, device=device)
    _lib.check("usv_contour_descriptors",
               lib.usv_contour_descriptors(d_pts.data_ptr(), d_off.data_ptr(), n, desc.data_ptr(), _stream(stream)))
    return desc[:n]


def contour_pair_scores(desc_a: torch.Tensor, desc_b: torch.Tensor, stream=None) -> torch.Tensor:
    """(n_a, n_b) float64 device tensor of matchShapes-I1 + |area ratio| scores."""
    lib = _lib.load()
    for t in (desc_a, desc_b):
        if not (t.is_cuda and t.dtype == torch.float64 and t.dim() == 2 and t.shape[1] == DESC and t.is_contiguous()):
            raise ValueError("descriptors must be contiguous (n, 8) float64 CUDA (HIP) tensors")
    n_a, n_b = desc_a.shape[0], desc_b.shape[0]
    scores = torch.empty((n_a, n_b), dtype=torch.float64, device=desc_a.device)
    _lib.check("usv_contour_pair_scores",
               lib.usv_contour_pair_scores(desc_a.data_ptr(), n_a, desc_b.data_ptr(), n_b, scores.data_ptr(),
                                           _stream(stream)))
    return scores


class ContourMatcherGPU:
    """usv_contour_matcher (include/usv.h): GenerateMatchingList on the device from host contour sets,
    selection and in-order compaction included, for up to max_contours contours and max_points points
    per set (pinned staging and device buffers allocated once, on the current HIP device).  The C matcher
    serves one call at a time (include/usv.h); a lock serialises callers that share this object (the
    module-level GenerateMatchingListGPU cache)."""

    def __init__(self, max_contours: int = 512, max_points: int = 1 << 16):
        import ctypes
        import threading
        self._ct = ctypes
        self._lock = threading.Lock()
        self.lib = _lib.load()
        self.max_contours, self.max_points = max_contours, max_points
        h = ctypes.c_void_p()
        _lib.check("usv_contour_matcher_create", self.lib.usv_contour_matcher_create(max_contours, max_points,
                                                                                     ctypes.byref(h)))
        self.handle = h
        self._out = (_lib.usv_match * 1)()

    def close(self):
        if self.handle:
            _lib.check("usv_contour_matcher_destroy", self.lib.usv_contour_matcher_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fits(self, n_a: int, n_b: int, p_a: int, p_b: int) -> bool:
        return max(n_a, n_b) <= self.max_contours and max(p_a, p_b) <= self.max_points

    def match_flat(self, pa, oa, pb, ob):
        """Flattened int32 sets (as usv_generate_matching_list) -> ctypes usv_match array, count.  The array
        is this object's output buffer: valid until its next call."""
        with self._lock:
            return self._match_flat(pa, oa, pb, ob)

    def _match_flat(self, pa, oa, pb, ob):
        ct = self._ct
        n_a, n_b = len(oa) - 1, len(ob) - 1
        cap = max(1, n_a * n_b)
        if len(self._out) < cap:
            self._out = (_lib.usv_match * cap)()
        n = ct.c_int(0)
        ip = ct.POINTER(ct.c_int)
        _lib.check("usv_generate_matching_list_gpu", self.lib.usv_generate_matching_list_gpu(
            self.handle, pa.ctypes.data_as(ip), oa.ctypes.data_as(ip), n_a, pb.ctypes.data_as(ip),
            ob.ctypes.data_as(ip), n_b, self._out, cap, ct.byref(n)))
        return self._out, n.value

    def __call__(self, contours_l, contours_r):
        pa, oa = _flatten(contours_l)
        pb, ob = _flatten(contours_r)
        with self._lock:  # the list is built before the output buffer can be reused
            out, n = self._match_flat(pa, oa, pb, ob)
            return [(out[k].left_index, out[k].right_index, out[k].match_value) for k in range(n)]


_MATCHERS: dict[int, ContourMatcherGPU] = {}
_MATCHERS_LOCK = __import__("threading").Lock()
# The matcher holds max_contours^2 x 16 B of pinned host memory and twice that on the device (score rows and
# the compacted list): the per-device cache keeps one of at most _CACHE_MAX_CONTOURS contours (4096: 268 MB
# pinned); larger sets take the descriptor + score launches with the selection done by torch on the device
# (n^2 x 8 B of scores instead of a per-call matcher's n^2 x 48 B of pinned host and device buffers).
_CACHE_MAX_CONTOURS = 4096
_MATCHER_MAX_CONTOURS = 16384  # usv_contour_matcher_create's limit


def _select_on_device(contours_l, contours_r, dev):
    """contour_descriptors + contour_pair_scores, then v < 0.75 (NaN fails) kept in row-major order."""
    scores = contour_pair_scores(contour_descriptors(contours_l, dev), contour_descriptors(contours_r, dev))
    keep = scores < 0.75
    ij = torch.nonzero(keep)  # row-major: i-major, j-minor as P/Main.cpp:408-420
    vals = scores[keep]
    ij, vals = ij.cpu().tolist(), vals.cpu().tolist()
    return [(i, j, v) for (i, j), v in zip(ij, vals)]


def GenerateMatchingListGPU(contours_l, contours_r, device="cuda", stream=None):
    """Contours as lists of (x, y) int points -> list[(i, j, score)] with score < 0.75 (NaN dropped), i-major
    then j-minor like GenerateMatchingList (P/Main.cpp:403-426), through the device matcher
    (usv_generate_matching_list_gpu: one H2D copy, descriptors + selection on the device, one D2H copy).
    `stream` is unused: the matcher owns its stream and returns host results."""
    del stream
    if not contours_l or not contours_r:  # P/Main.cpp:405
        return []
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    n = max(len(contours_l), len(contours_r))
    p = max(sum(len(c) for c in contours_l), sum(len(c) for c in contours_r))
    if n > _CACHE_MAX_CONTOURS:
        # a matcher for one call would pin n^2 x 16 B on the host and twice that on the device (4.3 GB and
        # 8.6 GB at n = 16384), allocated and freed per call; the descriptor + score launches with the
        # selection on the device need only the n^2 x 8 B score matrix
        with torch.cuda.device(idx):
            return _select_on_device(contours_l, contours_r, torch.device("cuda", idx))
    with _MATCHERS_LOCK:
        m = _MATCHERS.get(idx)
        if m is None or not m.fits(n, n, p, p):
            # (a replaced matcher is freed when the last caller still using it drops it)
            with torch.cuda.device(idx):
                m = ContourMatcherGPU(max(512, n), max(1 << 16, p))
            _MATCHERS[idx] = m
    return m(contours_l, contours_r)

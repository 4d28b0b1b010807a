"""Batched contour matcher on the GPU.

``GenerateMatchingListGPU`` returns what ``GenerateMatchingList``
(P/Main.cpp:403-426, host restatement in csrc/host/matching.cpp) returns --
(i, j, v) for every pair with v < 0.75, i-major then j-minor -- but computes
each contour's Hu-moment I1 terms and area once on the device
(``usv_contour_descriptors``) and all N×M scores in one launch
(``usv_contour_pair_scores``), instead of the reference's per-pair
recomputation.  The threshold/compaction of the N×M score matrix runs on the
host after one device-to-host copy (order-preserving, tiny).

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


def GenerateMatchingListGPU(contours_l, contours_r, device="cuda", stream=None):
    """Contours as lists of (x, y) int points -> list[(i, j, score)] with score < 0.75 (NaN dropped)."""
    if not contours_l or not contours_r:  # P/Main.cpp:405
        return []
    s = contour_pair_scores(contour_descriptors(contours_l, device, stream),
                            contour_descriptors(contours_r, device, stream), stream).cpu().numpy()
    ii, jj = np.nonzero(s < 0.75)  # row-major: i-major, j-minor
    return [(int(i), int(j), float(s[i, j])) for i, j in zip(ii, jj)]

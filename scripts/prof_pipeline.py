#!/usr/bin/env python3
"""Run each pipeline stage 20x at 1920x1080 (for rocprofv3 --kernel-trace --stats)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unsynchronized_stereo_vision_proj325_amd.preproc import ABSDiffSearch, FramePrep, FramePrepPair  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair, synthetic_calibration  # noqa

dev = torch.device("cuda:0")
W, H = 1920, 1080
rng = np.random.default_rng(0)
cl, cr = synthetic_calibration(W, H, seed=1)
rl, rr = Rectifier(*cl, (W, H), device=dev), Rectifier(*cr, (W, H), device=dev)
# the opt-in LDS-tiled packed remap beside the direct default: both kernels in the same trace
dl, dr = Rectifier(*cl, (W, H), device=dev, tiled=True), Rectifier(*cr, (W, H), device=dev, tiled=True)
src = [torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev) for _ in range(2)]
prep = FramePrep(dev)
gray = torch.from_numpy(rng.integers(0, 256, (H, W), dtype=np.uint8)).to(dev)
prev = torch.from_numpy(rng.integers(0, 256, (H, W), dtype=np.uint8)).to(dev)
pair = FramePrepPair(dev)
for _ in range(int(os.environ.get("PP_ITERS", "20"))):
    ol, orr = rectify_pair(rl, rr, src[0], src[1])
    rectify_pair(dl, dr, src[0], src[1])
    hsv, bgr, g = prep(ol)
    m, _ = ABSDiffSearch(gray, prev)
    pair(ol, orr)
    pair.rectify_prep(rl, rr, src[0], src[1])
torch.cuda.synchronize()
print("ok")

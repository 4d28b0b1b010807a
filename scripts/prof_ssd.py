#!/usr/bin/env python3
"""Run an SSD kernel N times back to back at config C (1920x1080, w = 11, D = 128) for rocprofv3 --kernel-trace /
--pmc passes (parity is tests/test_gpu_parity.py's and tests/test_ssd_matrix.py's job).

The launches are warm, as bench.py's `fallbacks.ssd_matrix` leg times them: first ~100 ms of the SAD matcher
(another kernel, so the trace's SSD statistics hold none of these clock-ramp launches; from idle the MI355X runs
its first ~20 ms of launches at lower clocks), then the SSD launches enqueued through a bound plan,
so the stream never drains between them.
    python scripts/prof_ssd.py [fast|matrix] [launches] [--cold]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher  # noqa: E402

W, H, D, w = 1920, 1080, 128, 11
args = [a for a in sys.argv[1:] if not a.startswith("--")]
kernel = args[0] if args else "fast"
n = int(args[1]) if len(args) > 1 else 300
rng = np.random.default_rng(5)
L = rng.integers(0, 256, (H, W), dtype=np.uint8)
R = np.roll(L, 17, axis=1) ^ rng.integers(0, 3, (H, W), dtype=np.uint8)
dev = torch.device("cuda:0")
Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
out = torch.empty((H, W), dtype=torch.uint8, device=dev)
ssd = StereoBlockMatcher(D, w, "ssd", kernel=kernel).bind(Lt, Rt, out_disp=out)
if "--cold" not in sys.argv:
    sad = StereoBlockMatcher(D, w).bind(Lt, Rt, out_disp=torch.empty_like(out))
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.1:
        for _ in range(16):
            sad()
        torch.cuda.synchronize()
    for _ in range(8):  # queue ahead of the SSD launches: no gap between the two kernels' streams of work
        sad()
for _ in range(n):
    ssd()
torch.cuda.synchronize()
print("ok")

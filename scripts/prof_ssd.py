#!/usr/bin/env python3
"""Run an SSD kernel 300x at config C (1920x1080, w = 11, D = 128) for rocprofv3 --kernel-trace / --pmc passes
(scripts/prof_kernel_ab.sh style A/Bs; parity is tests/test_gpu_parity.py's job).
    python scripts/prof_ssd.py [fast|matrix] [launches]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher  # noqa: E402

W, H, D, w = 1920, 1080, 128, 11
rng = np.random.default_rng(5)
L = rng.integers(0, 256, (H, W), dtype=np.uint8)
R = np.roll(L, 17, axis=1) ^ rng.integers(0, 3, (H, W), dtype=np.uint8)
dev = torch.device("cuda:0")
Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
ssd = StereoBlockMatcher(D, w, "ssd", kernel=sys.argv[1] if len(sys.argv) > 1 else "fast")
out = torch.empty((H, W), dtype=torch.uint8, device=dev)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 300):
    ssd.compute(Lt, Rt, out_disp=out)
torch.cuda.synchronize()
print("ok")

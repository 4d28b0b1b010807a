#!/usr/bin/env python3
"""Cold-cache launches of the block matcher for rocprofv3 PMC passes (HBM bytes per launch).

Between two launches a 512 MiB write evicts the XCD L2s and the 256 MiB Infinity Cache, so the
matcher's FETCH_SIZE / WRITE_SIZE per dispatch count the bytes it moves from and to HBM (with the
bench's back-to-back launches the inputs stay cached and the counters fall below the compulsory
bytes).  Usage: prof_cold.py W H D w [launches] [--no-distance]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.synthetic import synthetic_pair  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
W, H, D, w = (int(v) for v in args[:4])
n = int(args[4]) if len(args) > 4 else 10
with_dist = "--no-distance" not in sys.argv
dev = torch.device("cuda:0")
L, R, _ = synthetic_pair(W, H, D, pair_index=0, noise=2)
Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
m = StereoBlockMatcher(D, w)
disp = torch.empty((H, W), dtype=torch.uint8, device=dev)
dist = torch.empty((H, W), dtype=torch.float64, device=dev) if with_dist else None
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
for i in range(n):
    flush.fill_(i & 0xFF)
    m.compute(Lt, Rt, with_distance=with_dist, out_disp=disp, out_dist=dist)
torch.cuda.synchronize()
print(f"ok: {n} cold launches of {W}x{H} w={w} D={D}{' + distance' if with_dist else ''}")

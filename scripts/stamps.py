#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fast kernel from a USV_STAMPS=1 build.

    scripts/build_variant.sh stamps -DUSV_STAMPS=1 [-DUSV_DEV_ONLY_RAD=5 -DUSV_DEV_ONLY_NW=2]
    USV_LIB_PATH=$PWD/build_variants/stamps.so python scripts/stamps.py [--iters 20]
"""
import argparse
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher, _lib  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.synthetic import synthetic_pair  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--disparities", type=int, default=128)
ap.add_argument("--window", type=int, default=11)
a = ap.parse_args()
lib = _lib.load()
fn = lib.usv_debug_stamps
fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
L, R, _ = synthetic_pair(a.width, a.height, a.disparities, pair_index=0, noise=2)
Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
m = StereoBlockMatcher(a.disparities, a.window)
m.compute(Lt, Rt, with_distance=True)
torch.cuda.synchronize()
assert fn(buf, 1) == 0
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.iters):
    m.compute(Lt, Rt, with_distance=True)
e.record()
torch.cuda.synchronize()
assert fn(buf, 1) == 0
v = list(buf)
rows, waves, total = v[5], v[6], v[7]
names = ["dma_wait", "lword_wait", "chain_h_s", "keys_reduce", "flush"]
out = {"kernel_us": s.elapsed_time(e) / a.iters * 1e3, "waves_per_launch": waves / a.iters,
       "rows_per_wave": rows / waves, "cycles_per_wave": total / waves,
       "cycles_per_row": {n: v[i] / rows for i, n in enumerate(names)},
       "cycles_per_row_total": total / rows}
print(json.dumps(out, indent=1))

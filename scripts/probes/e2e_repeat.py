"""Probe (round 5): repeat bench.e2e_leg in one process and print each
repetition's depth-2 / depth-3 frame periods, to see how often a slow depth-3 measurement occurs."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
from bench import e2e_leg  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.synthetic import synthetic_pair  # noqa: E402

dev = torch.device("cuda:0")
L, R, _ = synthetic_pair(1920, 1080, 128, pair_index=1, noise=2)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    t = time.perf_counter()
    r = e2e_leg(dev, L, R, 128, 11, 20)
    print(i, {k: round(v["ms_per_frame"], 4) for k, v in r["by_depth"].items()}, "leg %.2f s" % (time.perf_counter() - t),
          flush=True)

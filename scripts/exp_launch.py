#!/usr/bin/env python3
"""Launch-overhead experiment (GPU box): wall time per step of config C with
(a) per-step event pairs, (b) one event pair around the region, (c) steps
alternating over two streams, (d) a HIP graph of 8 steps replayed."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.synthetic import synthetic_pair  # noqa: E402

dev = torch.device("cuda:0")
L, R, _ = synthetic_pair(1920, 1080, 128, pair_index=0, noise=2)
Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
m = StereoBlockMatcher(128, 11)
K = 200
disp = [torch.empty((1080, 1920), dtype=torch.uint8, device=dev) for _ in range(2)]
dist = [torch.empty((1080, 1920), dtype=torch.float64, device=dev) for _ in range(2)]
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def run(mode):
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    t0 = time.perf_counter()
    if mode == "graph":
        for _ in range(K // 8):
            g.replay()
    else:
        for i in range(K):
            b = i % 2
            s = streams[b] if mode == "2streams" else torch.cuda.current_stream()
            with torch.cuda.stream(s):
                if mode in ("per-step", "2streams"):
                    evs[i][0].record(s)
                m.compute(Lt, Rt, with_distance=True, out_disp=disp[b], out_dist=dist[b], stream=s)
                if mode in ("per-step", "2streams"):
                    evs[i][1].record(s)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e6
    kern = sum(a.elapsed_time(b) for a, b in evs) / K * 1e3 if mode in ("per-step", "2streams") else float("nan")
    print(f"{mode:10s} wall/step {wall:7.2f} us   event kernel {kern:7.2f} us", flush=True)


for mode in ("per-step", "none", "per-step", "none", "2streams", "2streams"):
    run(mode)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for i in range(3):
        m.compute(Lt, Rt, with_distance=True, out_disp=disp[i % 2], out_dist=dist[i % 2], stream=s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    for i in range(8):
        m.compute(Lt, Rt, with_distance=True, out_disp=disp[i % 2], out_dist=dist[i % 2], stream=s)
run("graph")
run("graph")

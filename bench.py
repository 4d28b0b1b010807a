#!/usr/bin/env python3
"""Headline benchmark: disparity-pixels/s of the SAD block matcher on MI355X.

Workload (BASELINE.json configs[2], "C"): 1920x1080 u8 synthetic rectified
pair, 11x11 SAD, 128 disparities, plus the fused per-pixel distance map (cm,
f64) -- one "step" = one pair through the hot path with inputs resident in
HBM.  N GPUs = weak scaling (config D at N=8): every rank owns one pair per
step (independent, no data-path collective) and rank 0 gathers the u8
disparity maps over RCCL (xGMI), overlapped with the next step's compute.
Consecutive steps are independent frames and alternate over two HIP streams
(--streams, default 2), so the tail of frame k's launch -- its last
workgroups, when most CUs are already idle -- overlaps the head of frame
k+1's, as a frame server keeps two frames in flight; ms_per_step is then
below the isolated launch time kernel_ms, which stays the roofline basis.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (driver, N > 1)

`--gpus N` must equal the launcher's WORLD_SIZE.  Without a launcher (no
WORLD_SIZE in the environment) and N > 1, bench.py starts the N ranks itself
(torch.distributed.run as a CHILD process, before anything touches the GPU)
and exits with its status; fewer than N visible GPUs is an error.  It never
reports a one-rank run for --gpus N > 1.

Prints ONE JSON line on rank 0 (the driver's contract) with "roofline" for
the dominant kernel (HBM algorithmic bytes / avg kernel time, HIP events on
the kernel's stream) and, at N=1, "cpu_baseline" (the C oracle's
multithreaded sliding-window variant on a bounded row band of the same pair).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from unsynchronized_stereo_vision_proj325_amd import StereoBlockMatcher  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.sharding import band_range, gather_disparity, pair_range  # noqa: E402
from unsynchronized_stereo_vision_proj325_amd.synthetic import synthetic_pair  # noqa: E402

# BASELINE.json's metric, verbatim (value = disparity-pixels/s; achieved HBM GB/s is roofline.achieved)
BASELINE_METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# 256 CU x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T lane-ops/s (32-bit VALU, MI355X_MICROARCH.md)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--disparities", type=int, default=128)
    p.add_argument("--window", type=int, default=11)
    p.add_argument("--no-distance", action="store_true", help="disparity map only (no fused distance map)")
    p.add_argument("--gather", choices=["overlap", "sync", "none"], default="overlap")
    p.add_argument("--split", choices=["pairs", "bands"], default="pairs",
                   help="N > 1: one pair per GPU (weak scaling, config D) or one frame split into row bands "
                        "with halos (strong scaling of config C, sharding.match_band)")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="CPU-baseline sample budget: warm-up + 5 timed runs share it (N=1 only)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--streams", type=int, default=2,
                   help="HIP streams the timed steps alternate over (consecutive frames are independent, so "
                        "with 2 one launch's tail overlaps the next launch's head)")
    p.add_argument("--no-parity", action="store_true",
                   help="skip the oracle parity checks after the timed region (profiling passes only)")
    p.add_argument("--extra-steps", type=int, default=20,
                   help="timed frames per extra leg (end-to-end, frame chain, generic fallbacks); 0 = skip")
    p.add_argument("--warm-ms", type=float, default=60.0,
                   help="after the W warmup steps, keep stepping (untimed) until this much wall time has passed: "
                        "the GPU raises its clocks only under sustained load (0 = off)")
    p.add_argument("--kernel-steps", type=int, default=50,
                   help="launches of the separate back-to-back pass after the timed region that gives "
                        "kernel_ms (HIP events around the pass only, queued behind as many untimed launches "
                        "so the host enqueues them all); 0 = use the timed region's span")
    p.add_argument("--pipeline-steps", type=int, default=50,
                   help="timed launches per pipeline leg (rectify / frame prep / mask); 0 = skip")
    return p.parse_args()


def _config_name(W, H, w, D) -> str:
    """BASELINE.json config letter for these dimensions (A..E), else "custom"."""
    return {(320, 240, 5, 32): "A", (640, 480, 7, 64): "B", (1920, 1080, 11, 128): "C",
            (3840, 2160, 15, 256): "E"}.get((W, H, w, D), "custom")


def profile_counters(workload_key: str):
    """Per-launch counters of the committed rocprofv3 run for this workload
    (profiles/counters.json, written by scripts/summarize_profile.py), or None."""
    path = os.path.join(ROOT, "profiles", "counters.json")
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path)).get(workload_key)
    except (OSError, ValueError):
        return None


def fast_kernel_name(W: int, D: int, w: int, pitch: int) -> str:
    """Which kernel the AUTO dispatch takes for this shape (csrc/usv_sad_fast.hip
    fast_path_supported / pair_path_supported / launch_fast), for labelling the roofline entry."""
    if 3 <= w <= 15 and w % 2 == 1 and 1 <= D <= 256 and W % 4 == 0 and W >= 48 and pitch % 4 == 0:
        if D % 2 == 0 and 16 < D <= 64 and 5 <= w <= 9:  # csrc/usv_sad_group.hip group_path_supported
            return f"sad_group_kernel<{(w - 1) // 2}, {2 if D > 32 else 4}>"
        if D > 64 and D % 2 == 0 and w >= 11:
            return f"sad_pair_kernel<{(w - 1) // 2}, {1 if D <= 128 else 2}>"
        nw = 1 if D <= 64 else (2 if D <= 128 else 4)
        return f"sad_fast_kernel<{(w - 1) // 2}, {nw}>"
    return "sad_generic_kernel"


def cpu_baseline(L: np.ndarray, R: np.ndarray, D: int, w: int, budget_s: float, runs: int = 5):
    """Oracle (oracle/sad_oracle.c sliding variant, all allowed cores) on a bounded row band of the
    same pair: one warm-up run, then the median of `runs` timed runs."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import load_oracle

    lib = load_oracle()
    H, W = L.shape
    cores = max(1, min(16, os.cpu_count() or 1))  # the GPU box's CPU share is 16
    out = np.zeros_like(L)

    def run(rows, reps=1):
        t0 = time.perf_counter()
        for _ in range(reps):
            rc = lib.usv_oracle_sad_sliding_rows(L.ctypes.data, R.ctypes.data, W, H, W, D, w, 0,
                                                 out.ctypes.data, W, 0, rows, cores)
            assert rc == 0
        return time.perf_counter() - t0

    # a run = `rows` rows of the pair, repeated `reps` times, sized so warm-up + `runs` runs fill the budget
    per_run = budget_s / (runs + 1)
    probe = max(cores, 16)
    t = run(probe)
    rows = int(min(H, max(probe, probe * per_run / max(t, 1e-6))))
    reps = 1
    if rows == H:
        reps = max(1, int(per_run / max(run(H), 1e-6)))
    run(rows, reps)  # warm-up
    times = [run(rows, reps) for _ in range(runs)]
    med = float(np.median(times))
    return {
        "value": reps * rows * W / med,
        "unit": "disparity-pixels/s",
        "cores": cores,
        "kind": "port",
        "sample": f"oracle sliding-window SAD, rows 0..{rows} of the {W}x{H} w={w} D={D} pair, {reps} time(s) per "
                  f"run ({reps * rows * W} output pixels per run), median of {runs} runs after one warm-up",
        "runs_s": times,
    }


def _oracle_dist_lut(lib) -> np.ndarray:
    """The oracle's 256-entry distance table (oracle/distance_oracle.c, P/DistanceCalculator.cpp:84)."""
    return np.array([lib.usv_oracle_distance_cm(d) for d in range(256)], dtype=np.float64)


def _mismatches(got_disp: np.ndarray, ref: np.ndarray, got_dist, lut: np.ndarray) -> dict:
    """Mismatch counts of one output against the oracle's disparity map: u8 disparity bytes, and the f64
    distance map bit for bit against lut[ref] (inf at d = 0 compares equal as bits)."""
    res = {"pixels": int(ref.size), "disparity_mismatches": int((got_disp != ref).sum())}
    if got_dist is not None:
        want = lut[ref.astype(np.int64)]
        res["distance_mismatches"] = int((got_dist.view(np.uint64) != want.view(np.uint64)).sum())
    return res


def parity_checks(dev, L: np.ndarray, R: np.ndarray, D: int, w: int, outputs, one_shots: bool) -> dict:
    """Checker, run after the timed region (never inside it): the timed kernel's own output buffers
    against the oracle (oracle/sad_oracle.c sliding variant, bit-exact with the naive definition) on
    the same pair, plus, with one_shots, full-size configs A, B, E and config C SSD through
    StereoBlockMatcher and config D (batch of 8) through the C-ABI sharded engine (usv_batch_sharded,
    one GPU).  Distance maps are compared bit for bit with the oracle's table at the oracle's
    disparity (P/DistanceCalculator.cpp:84).  Returns per-config mismatch counts; "ok" is the AND."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import load_oracle, oracle_sad

    threads = max(1, min(16, os.cpu_count() or 1))
    lib = load_oracle()
    lut = _oracle_dist_lut(lib)
    H, W = L.shape
    t0 = time.perf_counter()
    ref = oracle_sad(L, R, D, w, "sad", "sliding", threads)
    res = {}
    for i, (disp_t, dist_t) in enumerate(outputs):
        got = disp_t.cpu().numpy()
        res[f"timed_buffer{i}"] = _mismatches(got, ref, dist_t.cpu().numpy() if dist_t is not None else None, lut)
    if one_shots:
        for name, (cW, cH, cD, cw, metric) in {"A": (320, 240, 32, 5, "sad"), "B": (640, 480, 64, 7, "sad"),
                                              "C_ssd": (W, H, D, w, "ssd"),
                                              "E": (3840, 2160, 256, 15, "sad")}.items():
            cL, cR, _ = synthetic_pair(cW, cH, cD, pair_index=3, noise=2)
            m = StereoBlockMatcher(cD, cw, metric)
            disp, dist_map = m.compute(torch.from_numpy(cL).to(dev), torch.from_numpy(cR).to(dev), with_distance=True)
            torch.cuda.synchronize()
            cref = oracle_sad(cL, cR, cD, cw, metric, "sliding", threads)
            res[name] = {"workload": f"{cW}x{cH} w={cw} D={cD} {metric.upper()}",
                         **_mismatches(disp.cpu().numpy(), cref, dist_map.cpu().numpy(), lut)}
            del disp, dist_map
        from unsynchronized_stereo_vision_proj325_amd.sharding import ShardedMatcher
        B = 8
        pairs = [synthetic_pair(W, H, D, pair_index=16 + i, noise=2) for i in range(B)]
        bL = np.stack([p[0] for p in pairs])
        bR = np.stack([p[1] for p in pairs])
        eng = ShardedMatcher([dev.index if dev.index is not None else 0], B, W, H, D, w)
        try:
            bd, bx = eng.run(bL, bR, with_distance=True)
        finally:
            eng.close()
        tot = {"pixels": 0, "disparity_mismatches": 0, "distance_mismatches": 0}
        for i in range(B):
            mm = _mismatches(bd[i], oracle_sad(bL[i], bR[i], D, w, "sad", "sliding", threads), bx[i], lut)
            for k in tot:
                tot[k] += mm[k]
        res["D"] = {"workload": f"batch of {B} x {W}x{H} w={w} D={D} SAD through usv_batch_sharded (1 GPU)", **tot}
    bad = sum(v.get("disparity_mismatches", 0) + v.get("distance_mismatches", 0) for v in res.values())
    res["ok"] = bad == 0
    res["checker"] = (f"oracle/sad_oracle.c sliding variant ({threads} threads) and oracle/distance_oracle.c "
                      "table; outside the timed region")
    res["check_s"] = time.perf_counter() - t0
    return res


def cpu_naive_configs() -> dict:
    """The naive single-thread oracle (definition-level triple loop, oracle/sad_oracle.c) on configs A
    and B in full: median of 3 runs after a warm-up."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import load_oracle

    lib = load_oracle()
    res = {}
    for name, (W, H, D, w) in {"A": (320, 240, 32, 5), "B": (640, 480, 64, 7)}.items():
        L, R, _ = synthetic_pair(W, H, D, pair_index=0, noise=2)
        out = np.zeros_like(L)

        def run():
            t0 = time.perf_counter()
            assert lib.usv_oracle_sad_naive(L.ctypes.data, R.ctypes.data, W, H, W, D, w, 0, out.ctypes.data, W) == 0
            return time.perf_counter() - t0

        run()
        times = [run() for _ in range(3)]
        med = float(np.median(times))
        res[name] = {"workload": f"{W}x{H} w={w} D={D}", "ms_per_pair": med * 1e3,
                     "value": W * H / med, "unit": "disparity-pixels/s", "cores": 1, "kind": "port",
                     "runs_s": times}
    return res


_BUSY = []


def _busy_work(n: int, stream) -> None:
    """Enqueue n full-chip elementwise passes over 64 MB (~20-30 us each): they hold the stream while the
    host enqueues the timed launches behind them and keep the clocks up (a one-wave spin kernel let the
    GPU lower them)."""
    if not _BUSY:
        _BUSY.extend([torch.zeros(16 << 20, dtype=torch.float32, device=stream.device) for _ in range(2)])
    a, b = _BUSY
    with torch.cuda.stream(stream):
        for _ in range(n):
            torch.add(a, 1.0, out=b)


def time_launches(fn, steps: int, stream, warm_ms: float = 10.0, graph_ok: bool = True,
                  preload: str = "busy") -> float:
    """Average duration (us) of `fn()` over `steps` back-to-back launches, HIP events on `stream`.
    After `warm_ms` of untimed launches (the GPU lowers its clocks whenever it idles) the stream is
    preloaded so that the host's enqueue time is hidden, then the launches are enqueued between two
    events: the interval is GPU time, without enqueue gaps or an idle-lowered clock.  preload "busy":
    full-chip elementwise passes over 64 MB (for kernels shorter than a Python launch); "self": `steps`
    untimed launches of fn itself (for kernels longer than a launch -- the matcher: memory-bound busy
    work ahead of it let the core clock sag, 63.6 vs 56.8 us).  Round 2 held the stream with a one-wave
    spin kernel, during which the clocks dropped (62.2 vs 59.0 us per launch at config C); a HIP-graph
    replay adds ~5 us per node to few-us kernels."""
    del graph_ok  # (kept for callers; no capture is used)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    while (time.perf_counter() - t_w) * 1e3 < warm_ms:
        for _ in range(8):
            fn()
        torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if preload == "self":
        with torch.cuda.stream(stream):
            for _ in range(steps):
                fn()
    else:
        _busy_work(max(8, steps), stream)  # >= ~25 us of GPU work per launch the host must enqueue
    with torch.cuda.stream(stream):
        start.record(stream)
        for _ in range(steps):
            fn()
        end.record(stream)
    end.synchronize()
    return start.elapsed_time(end) / steps * 1e3


def pipeline_legs(dev, W: int, H: int, steps: int) -> dict:
    """The per-frame stages around the block matcher, config C geometry,
    synthetic BGR frames and calibration; each leg's roofline is HBM (algorithmic bytes / avg launch)."""
    from unsynchronized_stereo_vision_proj325_amd.preproc import ABSDiffSearch, FramePrep, FramePrepPair
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair, synthetic_calibration

    rng = np.random.default_rng(7)
    cl, cr = synthetic_calibration(W, H, seed=1)
    rl, rr = Rectifier(*cl, (W, H), device=dev), Rectifier(*cr, (W, H), device=dev)  # packed maps (4 B/px)
    ul, ur = (Rectifier(*cl, (W, H), device=dev, packed=False),
              Rectifier(*cr, (W, H), device=dev, packed=False))  # OpenCV's map pair (6 B/px)
    mb = 4 if rl.pmap is not None else 6
    src_l = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    src_r = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    out_l, out_r = torch.empty_like(src_l), torch.empty_like(src_r)
    prep = FramePrep(dev)
    hsv, bgr2, gray = torch.empty_like(src_l), torch.empty_like(src_l), torch.empty((H, W), dtype=torch.uint8,
                                                                                   device=dev)
    prev = torch.from_numpy(rng.integers(0, 256, (H, W), dtype=np.uint8)).to(dev)
    mask = torch.empty_like(prev)
    s = torch.cuda.current_stream()
    px = W * H
    legs = {
        # 2 cameras x (packed map 4 B, source 3 B, output 3 B) per pixel
        "rectify_pair_bgr": (lambda: rectify_pair(rl, rr, src_l, src_r, out_l, out_r), 2 * px * (mb + 3 + 3)),
        # the same through OpenCV's CV_16SC2 + CV_16UC1 map pair (map 4 + 2 B)
        "rectify_pair_bgr_map_pair": (lambda: rectify_pair(ul, ur, src_l, src_r, out_l, out_r), 2 * px * (6 + 3 + 3)),
        # V histogram (3 in) + BGR2HSV/equalize/HSV2BGR/gray (3 in, 3 + 3 + 1 out), one camera
        "frame_prep": (lambda: prep(out_l, hsv, bgr2, gray), px * (3 + 3 + 7)),
        # absdiff + threshold + erode + dilate: gray + prev in, mask out
        "motion_mask": (lambda: ABSDiffSearch(gray, prev, out=mask), px * 3),
    }
    pair = FramePrepPair(dev)
    pouts = [torch.empty_like(src_l) for _ in range(4)] + [torch.empty((H, W), dtype=torch.uint8, device=dev)
                                                          for _ in range(2)]
    # both cameras' frame prep in two launches (usv_frame_prep_pair_u8)
    legs["frame_prep_pair"] = (lambda: pair(out_l, out_r, outs=pouts), 2 * px * (3 + 3 + 7))
    # the whole per-frame stage of the pair in two launches (usv_rectify_prep_pair_u8): rectify + HSV +
    # histogram (4 packed map + 3 src + 3 hsv), then equalize / HSV2BGR / gray (3 + 3 + 3 + 1), per camera
    legs["rectify_prep_pair"] = (lambda: pair.rectify_prep(rl, rr, src_l, src_r, outs=pouts),
                                 2 * px * (mb + 6 + 10))
    # Size-matched copy roof: a device-to-device copy moving the same bytes (half read, half written),
    # the rate a stream of this size actually reaches (launch ramp and tail included; 8 TB/s is not
    # reachable at tens of MB: profiles/probes_r03/stream_probe_r03.txt).
    cbuf = torch.empty(max(n for _, n in legs.values()), dtype=torch.uint8, device=dev)
    res = {}
    for name, (fn, nbytes) in legs.items():
        us = time_launches(fn, steps, s)
        gbs = nbytes / (us * 1e-6) / 1e9
        half = nbytes // 2
        src_c, dst_c = cbuf[:half], cbuf[half:2 * half]
        copy_us = time_launches(lambda: dst_c.copy_(src_c), steps, s)
        res[name] = {"us": us, "bytes": nbytes, "achieved_GBs": gbs, "frac_hbm": gbs / HBM_PEAK_GBS,
                     "copy_us_same_bytes": copy_us, "frac_of_copy": copy_us / us}
    return res


def spawn_ranks(n: int, need_gpus: bool) -> int:
    """Run this script as N ranks under torch.distributed.run and return its exit status.  The
    launcher is a fresh child process (subprocess, never an exec of this one), so it is legal even
    if torch.cuda.device_count() initialised the HIP runtime here (it may: without amdsmi PyTorch
    counts with hipGetDeviceCount); each rank re-checks WORLD_SIZE against the GPUs it sees."""
    import socket
    import subprocess
    if need_gpus:
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr)
            return 2
    with socket.socket() as sock:
        sock.bind(("127.0.0.1", 0))
        port = sock.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.run(cmd).returncode


def plumbing_rehearsal(a, world: int, rank: int) -> None:
    """USV_BENCH_PLUMBING=1: the N-rank launch contract on CPU (gloo), no GPU and no kernel -- rank
    spawn, the barriers around the timed region, max-over-ranks timing and the rank-0 JSON line.
    Its record carries value null: it measures nothing."""
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        pass
    if world > 1:
        dist.barrier()
    t = torch.tensor([time.perf_counter() - t0, float(rank)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": BASELINE_METRIC, "value": None, "unit": "disparity-pixels/s", "n_gpus": world,
                          "steps": a.steps, "warmup": a.warmup, "ms_per_step": None, "higher_is_better": True,
                          "scaling": "weak", "vs_baseline": None, "dtype": "u8",
                          "data": "plumbing rehearsal: no GPU, no kernel (USV_BENCH_PLUMBING=1)",
                          "config": {"workload": "none", "parallelism": f"{world} gloo ranks"},
                          "max_rank_seen": int(t[1])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def e2e_leg(dev, L: np.ndarray, R: np.ndarray, D: int, w: int, steps: int) -> dict:
    """PCIe-inclusive frame rate through the streaming engine (usv_frame_stream_*, csrc/usv_stream.hip):
    host pair in pinned staging -> H2D -> match -> u8 disparity D2H, `depth` frames in flight so the
    copies of neighbouring frames overlap the kernel (the reference's caller hands over host frames,
    P/Main.cpp:876-921).  Beside it the serialised per-frame form (one stream, synchronised per frame,
    f64 distance map shipped back) that round 2 reported.  Never the headline value."""
    from unsynchronized_stereo_vision_proj325_amd.streaming import FrameStream, expand_distance

    H, W = L.shape
    out = {}
    for depth in (2, 3):  # (depth 4 measured slower than 3 in rounds 3-5: DESIGN.md section 7)
        fs = FrameStream(W, H, D, w, depth=depth)
        # frames already in each slot's pinned staging (a camera driver would DMA them there)
        staged = []
        for _ in range(depth):
            sl, sr = fs.next_inputs()
            sl[:] = L
            sr[:] = R
            t = fs.submit(sl, sr)
            staged.append(t)
        for t in staged:
            fs.wait(t)
            fs.release(t)

        def run(n):
            pending = []
            for _ in range(n):
                if len(pending) == depth:
                    t = pending.pop(0)
                    fs.wait(t)
                    fs.release(t)
                sl, sr = fs.next_inputs()
                pending.append(fs.submit(sl, sr))
            for t in pending:
                fs.wait(t)
                fs.release(t)

        # copy engines and clocks settle over the first few dozen frames (probe: 0.16 ms per frame for the
        # first ~100 at depth 3, 0.113 after): 64 warm frames, then the median of three timed windows
        run(64)
        n = max(steps, 50)
        win = []
        for _ in range(3):
            t0 = time.perf_counter()
            run(n)
            win.append((time.perf_counter() - t0) / n)
        dt = float(np.median(win))
        out[f"depth{depth}"] = {"ms_per_frame": dt * 1e3, "value": W * H / dt, "frames": 3 * n,
                                "windows_ms": [round(x * 1e3, 4) for x in win]}
        fs.close()
    best = min(out, key=lambda k: out[k]["ms_per_frame"])
    # a frame-rate consumer expands into the same host map every frame (persistent workers, pages already
    # mapped): median of 20 after 3 warm calls
    disp = np.random.default_rng(3).integers(0, D, (H, W), dtype=np.uint8)
    host_map = np.empty((H, W), dtype=np.float64)
    for _ in range(3):
        expand_distance(disp, threads=16, out=host_map)
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        expand_distance(disp, threads=16, out=host_map)
        ts.append(time.perf_counter() - t0)
    expand_ms = float(np.median(ts)) * 1e3

    matcher = StereoBlockMatcher(D, w)
    hl, hr = torch.from_numpy(L).pin_memory(), torch.from_numpy(R).pin_memory()
    dl, dr = torch.empty((H, W), dtype=torch.uint8, device=dev), torch.empty((H, W), dtype=torch.uint8, device=dev)
    hd = torch.empty((H, W), dtype=torch.uint8).pin_memory()
    hx = torch.empty((H, W), dtype=torch.float64).pin_memory()
    dd, dx = torch.empty_like(dl), torch.empty((H, W), dtype=torch.float64, device=dev)

    def frame():
        dl.copy_(hl, non_blocking=True)
        dr.copy_(hr, non_blocking=True)
        matcher.compute(dl, dr, with_distance=True, out_disp=dd, out_dist=dx)
        hd.copy_(dd, non_blocking=True)
        hx.copy_(dx, non_blocking=True)
        torch.cuda.current_stream().synchronize()

    for _ in range(3):
        frame()
    t0 = time.perf_counter()
    for _ in range(steps):
        frame()
    ser = (time.perf_counter() - t0) / steps
    return {"ms_per_frame": out[best]["ms_per_frame"], "value": out[best]["value"], "unit": "disparity-pixels/s",
            "depth": int(best[5:]), "by_depth": out, "bytes_h2d": 2 * W * H, "bytes_d2h": W * H,
            "host_distance_expand_ms_16_threads": expand_ms,
            "serial_fused_f64": {"ms_per_frame": ser * 1e3, "value": W * H / ser, "bytes_d2h": 9 * W * H,
                                 "note": "H2D + fused matcher + D2H of u8 and f64 maps, one stream, "
                                         "synchronised per frame (round-2 e2e leg)"},
            "note": "streaming engine: pinned host pair -> H2D -> match -> u8 disparity D2H, frames in flight "
                    "overlap; PCIe-inclusive, not the headline"}


def frame_chain_leg(dev, W: int, H: int, D: int, w: int, steps: int) -> dict:
    """The real per-frame chain on the device: rectify both BGR frames (one launch) -> frame prep
    of each camera (HSV, equalizeHist, BGR, gray) -> SAD block match of the rectified gray pair ->
    fused distance map (P/Main.cpp:913-921 then the north-star matcher), synthetic calibration."""
    from unsynchronized_stereo_vision_proj325_amd.preproc import FramePrep
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair, synthetic_calibration

    rng = np.random.default_rng(11)
    cl, cr = synthetic_calibration(W, H, seed=2)
    rl, rr = Rectifier(*cl, (W, H), device=dev), Rectifier(*cr, (W, H), device=dev)  # packed maps (4 B/px)
    ul, ur = (Rectifier(*cl, (W, H), device=dev, packed=False),
              Rectifier(*cr, (W, H), device=dev, packed=False))  # OpenCV's map pair (6 B/px)
    mb = 4 if rl.pmap is not None else 6
    src_l = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    src_r = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    rect_l, rect_r = torch.empty_like(src_l), torch.empty_like(src_r)
    pl, pr = FramePrep(dev), FramePrep(dev)
    bufs = [(torch.empty_like(src_l), torch.empty_like(src_l), torch.empty((H, W), dtype=torch.uint8, device=dev))
            for _ in range(2)]
    disp = torch.empty((H, W), dtype=torch.uint8, device=dev)
    dist = torch.empty((H, W), dtype=torch.float64, device=dev)
    matcher = StereoBlockMatcher(D, w)

    def frame():
        rectify_pair(rl, rr, src_l, src_r, rect_l, rect_r)
        pl(rect_l, *bufs[0])
        pr(rect_r, *bufs[1])
        matcher.compute(bufs[0][2], bufs[1][2], with_distance=True, out_disp=disp, out_dist=dist)

    us = time_launches(frame, steps, torch.cuda.current_stream(), preload="self")
    return {"us_per_frame": us, "value": W * H / (us * 1e-6), "unit": "disparity-pixels/s",
            "stages": "rectify pair (BGR) -> frame prep x2 -> SAD w=%d D=%d -> distance map" % (w, D),
            "launches_per_frame": 1 + 2 * 2 + 1}


def frame_chain_fused_leg(dev, W: int, H: int, D: int, w: int, steps: int) -> dict:
    """The per-frame chain with the fused stage: usv_rectify_prep_pair_u8 (rectify + HSV + histogram of
    both cameras, then equalize / HSV2BGR / gray of both) -> SAD block match -> distance map: three
    launches per frame instead of six.  Checked against the six-launch chain on the same input."""
    from unsynchronized_stereo_vision_proj325_amd.preproc import FramePrep, FramePrepPair
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, rectify_pair, synthetic_calibration

    rng = np.random.default_rng(11)
    cl, cr = synthetic_calibration(W, H, seed=2)
    rl, rr = Rectifier(*cl, (W, H), device=dev), Rectifier(*cr, (W, H), device=dev)  # packed maps (4 B/px)
    ul, ur = (Rectifier(*cl, (W, H), device=dev, packed=False),
              Rectifier(*cr, (W, H), device=dev, packed=False))  # OpenCV's map pair (6 B/px)
    mb = 4 if rl.pmap is not None else 6
    src_l = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    src_r = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    pair = FramePrepPair(dev)
    outs = [torch.empty_like(src_l) for _ in range(4)] + [torch.empty((H, W), dtype=torch.uint8, device=dev)
                                                         for _ in range(2)]
    disp = torch.empty((H, W), dtype=torch.uint8, device=dev)
    dist = torch.empty((H, W), dtype=torch.float64, device=dev)
    matcher = StereoBlockMatcher(D, w)

    def frame():
        pair.rectify_prep(rl, rr, src_l, src_r, outs=outs)
        matcher.compute(outs[4], outs[5], with_distance=True, out_disp=disp, out_dist=dist)

    frame()
    torch.cuda.synchronize()
    got = disp.clone()
    rect_l, rect_r = torch.empty_like(src_l), torch.empty_like(src_r)
    rectify_pair(rl, rr, src_l, src_r, rect_l, rect_r)
    gl = FramePrep(dev)(rect_l)[2]
    gr = FramePrep(dev)(rect_r)[2]
    same = bool(torch.equal(got, matcher.compute(gl, gr)))
    us = time_launches(frame, steps, torch.cuda.current_stream(), preload="self")
    return {"us_per_frame": us, "value": W * H / (us * 1e-6), "unit": "disparity-pixels/s",
            "stages": "rectify + HSV + hist (pair) -> equalize/HSV2BGR/gray (pair) -> SAD w=%d D=%d -> distance "
                      "map" % (w, D), "launches_per_frame": 3, "matches_six_launch_chain": same}


def time_alternating(fns, streams, steps: int, warm_ms: float = 10.0) -> float:
    """Average period (us) of `steps` calls that alternate over (fn, stream) pairs -- frame i runs fns[i % n]
    on streams[i % n] -- after `warm_ms` of warm calls and `steps` untimed calls preloaded ahead of the
    timed ones (as time_launches(preload="self")); HIP events on streams[0], joined with the others at
    the end."""
    n = len(fns)

    def run(k):
        for i in range(k):
            with torch.cuda.stream(streams[i % n]):
                fns[i % n]()

    run(2 * n)
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    while (time.perf_counter() - t_w) * 1e3 < warm_ms:
        run(4 * n)
        torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    run(steps)
    start.record(streams[0])
    run(steps)
    for s in streams[1:]:
        streams[0].wait_stream(s)
    end.record(streams[0])
    end.synchronize()
    return start.elapsed_time(end) / steps * 1e3


def frame_chain_overlap_leg(dev, W: int, H: int, D: int, w: int, steps: int) -> dict:
    """The fused three-launch chain (frame_chain_fused_leg) with consecutive frames alternating over two
    HIP streams, each with its own workspaces and outputs: frame k+1's memory-bound rectify / prep stage
    shares the chip with frame k's VALU-bound matcher, as a camera pipeline keeps two frames in flight.
    Each stream's maps are checked against the one-stream chain on the same input.  (This replaces the
    round-4 hipGraph form of the six-launch chain: replaying it was slower than eager, 112.9 vs 107.5 us,
    because the graph adds per-node overhead while the chain's cost is the kernels themselves.)"""
    from unsynchronized_stereo_vision_proj325_amd.preproc import FramePrepPair
    from unsynchronized_stereo_vision_proj325_amd.rectify import Rectifier, synthetic_calibration

    rng = np.random.default_rng(11)
    cl, cr = synthetic_calibration(W, H, seed=2)
    rl, rr = Rectifier(*cl, (W, H), device=dev), Rectifier(*cr, (W, H), device=dev)
    src_l = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    src_r = torch.from_numpy(rng.integers(0, 256, (H, W, 3), dtype=np.uint8)).to(dev)
    matcher = StereoBlockMatcher(D, w)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream(device=dev)]
    lanes = []
    for _ in streams:
        outs = [torch.empty_like(src_l) for _ in range(4)] + [torch.empty((H, W), dtype=torch.uint8, device=dev)
                                                             for _ in range(2)]
        lanes.append((FramePrepPair(dev), outs, torch.empty((H, W), dtype=torch.uint8, device=dev),
                      torch.empty((H, W), dtype=torch.float64, device=dev)))

    def make(lane):
        pair, outs, disp, dist = lane

        def frame():
            pair.rectify_prep(rl, rr, src_l, src_r, outs=outs)
            matcher.compute(outs[4], outs[5], with_distance=True, out_disp=disp, out_dist=dist)
        return frame

    fns = [make(lane) for lane in lanes]
    us = time_alternating(fns, streams, steps)
    torch.cuda.synchronize()
    pair, outs, disp, dist = lanes[0]
    ref_pair = FramePrepPair(dev)
    ref_outs = [torch.empty_like(o) for o in outs]
    ref_pair.rectify_prep(rl, rr, src_l, src_r, outs=ref_outs)
    ref_disp, ref_dist = matcher.compute(ref_outs[4], ref_outs[5], with_distance=True)
    torch.cuda.synchronize()
    same = all(bool(torch.equal(l[2], ref_disp) and torch.equal(l[3].nan_to_num(), ref_dist.nan_to_num()))
               for l in lanes)
    return {"us_per_frame": us, "value": W * H / (us * 1e-6), "unit": "disparity-pixels/s", "streams": 2,
            "stages": "rectify + HSV + hist (pair) -> equalize/HSV2BGR/gray (pair) -> SAD w=%d D=%d -> distance "
                      "map; frames alternate over two streams" % (w, D),
            "matches_one_stream_chain": same}


def matcher_leg(dev, n: int = 150, max_pts: int = 120, runs: int = 5) -> dict:
    """The reference's contour matcher on the host beside the engine's forms:
    N = M = n blob contours of 12..max_pts points.  Times (median of `runs` after one warm-up, host
    core count stated): the oracle's GenerateMatchingList, which recomputes both contours' Hu moments
    and four contourArea calls per pair as P/Main.cpp:403-426 does (the reference's algorithm, single
    thread); the host restatement (usv_generate_matching_list: descriptors once per contour); the GPU
    form (GenerateMatchingListGPU: descriptors + N x M scores in two launches, points H2D and scores
    D2H included); and ResolveMatchList (P/Main.cpp:432-477, the "VERy slow" step of :1079) in the
    oracle and the host C++.  The lists are checked equal (host bit-exact, GPU scores to 1e-12)."""
    import ctypes
    import math
    import random

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import _flat, load_oracle, oracle_match
    from unsynchronized_stereo_vision_proj325_amd import _lib
    from unsynchronized_stereo_vision_proj325_amd.contours import ContourMatcherGPU, GenerateMatchingListGPU

    rng = random.Random(325)

    def blob():
        cx, cy, r = rng.randint(40, 600), rng.randint(40, 440), rng.randint(8, 60)
        ang = sorted(rng.uniform(0, 2 * math.pi) for _ in range(rng.randint(12, max_pts)))
        return [(int(cx + r * rng.uniform(0.7, 1.0) * math.cos(a)), int(cy + r * rng.uniform(0.7, 1.0) * math.sin(a)))
                for a in ang]

    A, B = [blob() for _ in range(n)], [blob() for _ in range(n)]
    ora, lib = load_oracle(), _lib.load()
    pa, oa = _flat(A)
    pb, ob = _flat(B)
    cap = n * n
    o_out = (oracle_match * cap)()
    h_out = (_lib.usv_match * cap)()
    nh = ctypes.c_int(0)
    ip = ctypes.POINTER(ctypes.c_int)

    def med(fn):
        fn()
        ts = []
        for _ in range(runs):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3

    n_o = [0]

    def oracle_gml():
        n_o[0] = ora.usv_oracle_generate_matching_list(pa.ctypes.data, oa.ctypes.data, n, pb.ctypes.data,
                                                       ob.ctypes.data, n, o_out)

    def host_gml():
        _lib.check("usv_generate_matching_list", lib.usv_generate_matching_list(
            pa.ctypes.data_as(ip), oa.ctypes.data_as(ip), n, pb.ctypes.data_as(ip), ob.ctypes.data_as(ip), n,
            h_out, cap, ctypes.byref(nh)))

    with torch.cuda.device(dev):
        dm = ContourMatcherGPU(max(512, n), max(1 << 16, int(oa[-1]), int(ob[-1])))
    gpu_res = [None, 0]

    def gpu_gml():  # usv_generate_matching_list_gpu on the same flattened host arrays as host_gml
        gpu_res[0], gpu_res[1] = dm.match_flat(pa, oa, pb, ob)

    list_res = [None]

    def gpu_list():  # the Python entry (flatten + device matcher + list of tuples)
        list_res[0] = GenerateMatchingListGPU(A, B, device=dev)

    t_oracle, t_host, t_gpu, t_gpu_list = med(oracle_gml), med(host_gml), med(gpu_gml), med(gpu_list)
    ref = [(o_out[i].left, o_out[i].right, o_out[i].value) for i in range(n_o[0])]
    host = [(h_out[i].left_index, h_out[i].right_index, h_out[i].match_value) for i in range(nh.value)]
    gpu = [(gpu_res[0][k].left_index, gpu_res[0][k].right_index, gpu_res[0][k].match_value)
           for k in range(gpu_res[1])]
    dm.close()
    same_list = [x[:2] for x in list_res[0]] == [x[:2] for x in gpu]
    same_host = host == ref
    same_gpu = len(gpu) == len(ref) and all(g[:2] == r[:2] and abs(g[2] - r[2]) <= 1e-12 * (1 + abs(r[2]))
                                            for g, r in zip(gpu, ref))
    m = len(ref)
    r_in = (oracle_match * max(m, 1))()
    for i, (l, r, v) in enumerate(ref):
        r_in[i].left, r_in[i].right, r_in[i].value = l, r, v
    r_out = (oracle_match * max(m, 1))()
    h_in = (_lib.usv_match * max(m, 1))()
    for i, (l, r, v) in enumerate(ref):
        h_in[i].left_index, h_in[i].right_index, h_in[i].match_value = l, r, v
    h_res = (_lib.usv_match * max(m, 1))()
    nr, nrh = [0], ctypes.c_int(0)

    def oracle_rml():
        nr[0] = ora.usv_oracle_resolve_match_list(r_in, m, r_out)

    def host_rml():
        _lib.check("usv_resolve_match_list", lib.usv_resolve_match_list(h_in, m, h_res, ctypes.byref(nrh)))

    t_ro, t_rh = med(oracle_rml), med(host_rml)
    same_rml = nr[0] == nrh.value and all(
        (r_out[i].left, r_out[i].right, r_out[i].value) == (h_res[i].left_index, h_res[i].right_index,
                                                             h_res[i].match_value) for i in range(nr[0]))
    return {"workload": f"N = M = {n} contours of 12..{max_pts} points (seeded blobs), {m} pairs under 0.75",
            "cores": 1, "runs": runs,
            "generate_matching_list_ms": {"reference_algorithm_oracle": t_oracle, "host_cpp": t_host,
                                          "gpu": t_gpu, "gpu_python_list": t_gpu_list},
            "resolve_match_list_ms": {"reference_algorithm_oracle": t_ro, "host_cpp": t_rh},
            "speedup_host_vs_reference": t_oracle / t_host, "speedup_gpu_vs_reference": t_oracle / t_gpu,
            "lists_equal": {"host": same_host, "gpu": same_gpu, "gpu_python_list": same_list, "resolve": same_rml},
            "note": "single host thread for the CPU forms; gpu = usv_generate_matching_list_gpu on the same "
                    "flattened host arrays as host_cpp (one H2D copy, descriptor + selection launches that keep "
                    "v < 0.75 and compact each row in order, one D2H copy, rows concatenated on the host); "
                    "gpu_python_list = contours.GenerateMatchingListGPU (flatten + the same + a list of tuples); "
                    "resolve host_cpp = indexed form (per-index position lists), same output as the reference's scan"}


def fallback_legs(dev, L: np.ndarray, R: np.ndarray, D: int, w: int, steps: int) -> dict:
    """SSD and the paths off the fast SAD kernels: the SSD kernel (csrc/usv_sad_fast.hip
    ssd_fast_kernel, what AUTO runs for SSD at 11 <= w <= 15) at the headline config; the tiled
    sliding-window kernel (csrc/usv_sad_tiled.hip) for the same SSD and for SAD on a 1918-wide
    (W % 4 != 0) crop of the same pair; the direct-window generic kernel (csrc/usv_sad_generic.hip,
    O(D w^2) per pixel) beside them."""
    s = torch.cuda.current_stream()
    Lt, Rt = torch.from_numpy(L).to(dev), torch.from_numpy(R).to(dev)
    out = {}
    H, W = L.shape
    d1 = torch.empty_like(Lt)
    d2 = torch.empty((H, 1918), dtype=torch.uint8, device=dev)
    Lc, Rc = Lt[:, :1918], Rt[:, :1918]
    ssd = StereoBlockMatcher(D, w, "ssd", kernel="fast")
    us = time_launches(lambda: ssd.compute(Lt, Rt, out_disp=d1), steps * 8, s, preload="self")
    out["ssd_fast"] = {"workload": f"{W}x{H} w={w} D={D} SSD", "us": us, "value": W * H / (us * 1e-6),
                       "kernel": "ssd_fast_kernel (VALU)"}
    # the window cross term on the matrix cores (csrc/usv_ssd_mfma.hip): what AUTO runs for this SSD shape
    ssd = StereoBlockMatcher(D, w, "ssd", kernel="matrix")
    us = time_launches(lambda: ssd.compute(Lt, Rt, out_disp=d1), steps * 8, s, preload="self")
    out["ssd_matrix"] = {"workload": f"{W}x{H} w={w} D={D} SSD", "us": us, "value": W * H / (us * 1e-6),
                         "kernel": "ssd_mfma_kernel (v_mfma_i32_16x16x64_i8)",
                         "mfma_tops": 2.0 * 16 * 16 * 64 * (4 * (D // 16 + 1) * ((w + 3) // 4) * H * ((W + 63) // 64))
                         / (us * 1e-6) / 1e12}
    for kernel, n in (("tiled", steps * 8), ("generic", steps)):
        ssd = StereoBlockMatcher(D, w, "ssd", kernel=kernel)
        us = time_launches(lambda: ssd.compute(Lt, Rt, out_disp=d1), n, s, preload="self")
        out[f"ssd_{kernel}"] = {"workload": f"{W}x{H} w={w} D={D} SSD", "us": us, "value": W * H / (us * 1e-6)}
        sad = StereoBlockMatcher(D, w, kernel=kernel)
        us = time_launches(lambda: sad.compute(Lc, Rc, out_disp=d2), n, s, preload="self")
        out[f"sad_{kernel}_w1918"] = {"workload": f"1918x{H} (pitch {W}) w={w} D={D} SAD", "us": us,
                                      "value": 1918 * H / (us * 1e-6)}
    out["note"] = "AUTO runs ssd_matrix for SSD at w <= 13 and D = 32..160 step 32, ssd_fast at 11 <= w <= 15 " \
                  "otherwise, and the tiled kernel (vertical running sums, LDS-DMA row ring) for other SSD windows " \
                  "and for shapes outside the fast kernels (W % 4, W < 48, unaligned pitch or base); generic = one " \
                  "thread per pixel, direct window, only for w > 31; mfma_tops counts the MFMAs the matrix kernel " \
                  "issues (4 sub-tiles x (D/16 + 1) m-blocks x ceil(w/4) K-steps of 16x16x64 per 64-column tile-row: " \
                  "108 at D = 128, w = 11; edge triangles and the zero window column included)"
    return out


def main():
    a = parse()
    plumbing = os.environ.get("USV_BENCH_PLUMBING") == "1"
    # USV_BENCH_REHEARSE=1: several ranks on one GPU over gloo (a 1-GPU rehearsal of the N>1 code
    # path; use with --gather none, its numbers mean nothing)
    rehearse = os.environ.get("USV_BENCH_REHEARSE") == "1"
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(spawn_ranks(a.gpus, need_gpus=not (plumbing or rehearse)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if plumbing:
        plumbing_rehearsal(a, world, rank)
        return
    if rehearse:
        local %= torch.cuda.device_count()
    elif local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) visible")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    W, H, D, w = a.width, a.height, a.disparities, a.window
    with_dist = not a.no_distance
    # weak scaling: a batch of `world` independent pairs, pair i -> rank i (sharding.pair_range)
    bands = world > 1 and a.split == "bands"
    if bands:
        # strong scaling: every rank holds the frame, computes its row band from the halo'd input rows
        L, R, _ = synthetic_pair(W, H, D, pair_index=0, noise=2)
        y0, y1, i0, i1 = band_range(H, rank, world, w)
        band_w = max(pair_range(H, r, world)[1] - pair_range(H, r, world)[0] for r in range(world))
        rows = i1 - i0
    else:
        first, stop = pair_range(world, rank, world)
        assert stop - first == 1
        L, R, _ = synthetic_pair(W, H, D, pair_index=first, noise=2)
        y0, y1, i0, i1, rows = 0, H, 0, H, H
    Lt = torch.from_numpy(L).to(dev)[i0:i1]
    Rt = torch.from_numpy(R).to(dev)[i0:i1]
    matcher = StereoBlockMatcher(D, w)
    nbuf = max(2, a.streams)
    # (bands: one spare row so every rank can send band_w rows from y0 - i0 without a copy)
    disp_bufs = [torch.empty((1, rows + (1 if bands else 0), W), dtype=torch.uint8, device=dev) for _ in range(nbuf)]
    dist_bufs = [torch.empty((rows, W), dtype=torch.float64, device=dev) for _ in range(nbuf)] if with_dist else None
    recv = None
    if world > 1 and rank == 0 and a.gather != "none":
        shape = (band_w, W) if bands else (1, H, W)
        recv = [[torch.empty(shape, dtype=torch.uint8, device=dev) for _ in range(world)] for _ in range(nbuf)]
    stream = torch.cuda.current_stream()
    streams = [stream] + [torch.cuda.Stream(device=dev) for _ in range(max(1, a.streams) - 1)]
    pending = [None] * nbuf
    # one pre-marshalled C-ABI launcher per output buffer (StereoBlockMatcher.bind): a step enqueues its
    # match with one ctypes call, the same usv_sad_disparity_ex entry point compute() uses
    launch = [matcher.bind(Lt, Rt, out_disp=disp_bufs[b][0, :rows], out_dist=dist_bufs[b] if with_dist else None,
                           stream=streams[b % len(streams)]) for b in range(nbuf)]

    gathers = world > 1 and a.gather != "none"

    def step(i):
        b = i % nbuf
        if pending[b] is not None:  # the gather that last read this buffer must finish first
            with torch.cuda.stream(streams[b % len(streams)]):  # (wait() orders the current stream)
                pending[b].wait()
            pending[b] = None
        launch[b]()
        if gathers:
            with torch.cuda.stream(streams[b % len(streams)]):  # the gather is ordered behind this frame only
                collect(b)

    def collect(b):
        if bands and a.gather != "none":
            # rank 0 collects the bands (band_w rows from each; a rank's extra row is ignored)
            work = dist.gather(disp_bufs[b][0, y0 - i0:y0 - i0 + band_w], recv[b] if rank == 0 else None,
                               dst=0, async_op=True)
            if a.gather == "sync":
                work.wait()
            else:
                pending[b] = work
        elif world > 1 and a.gather != "none":
            # rank 0 collects every rank's u8 map over RCCL (xGMI); no concat copy
            work = gather_disparity(disp_bufs[b], world, dst=0, async_op=True,
                                    recv=recv[b] if rank == 0 else None, concat=False)
            if a.gather == "sync":
                work.wait()
            else:
                pending[b] = work

    torch.cuda.synchronize()
    t_w = time.perf_counter()
    for i in range(a.warmup):
        step(i)
    for b in range(nbuf):
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
    torch.cuda.synchronize()
    # pace of a step, from 16 more untimed steps (the W steps include first-launch costs)
    t_w = time.perf_counter()
    for i in range(16):
        step(a.warmup + i)
    for b in range(nbuf):
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
    torch.cuda.synchronize()
    per_step_s = (time.perf_counter() - t_w) / 16
    # Clock warm-up (untimed): from idle the MI355X runs the first ~20 ms of back-to-back launches at
    # lower clocks -- config C's kernel took 82.5 us per launch in a first 200-launch pass and 58.3 us in
    # the next (scripts/exp_launch.py, profiles/probes_r03/launch_modes_r03.txt).  A throughput number is
    # a sustained-load number, so the timed region starts after about --warm-ms of the same steps.  The
    # step count comes from the W warm-up steps' pace and is the same on every rank (MAX over ranks):
    # each step may carry a collective.
    warm_steps = int(min(20000, a.warm_ms * 1e-3 / max(per_step_s, 1e-6))) if a.warm_ms > 0 else 0
    if world > 1:
        t = torch.tensor([warm_steps], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        warm_steps = int(t.item())
    for i in range(warm_steps):
        step(a.warmup + 16 + i)
        if i % 64 == 63:
            torch.cuda.synchronize()  # (bounded queue depth)
    for b in range(nbuf):
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # The timed region carries no per-launch events (each event pair serialises the stream and costs
    # ~6 us of wall time, profiles/probes/launch_overhead_r01.txt): one event pair brackets the whole
    # region on the kernel's stream (span), and the per-launch kernel time comes from a separate
    # back-to-back pass after it (kernel_ms).
    span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    # (the device was synchronised above: the side streams are idle, nothing to order them behind)
    span[0].record(stream)
    for i in range(a.steps):
        step(i)
    t_enq = time.perf_counter()
    for extra in streams[1:]:
        stream.wait_stream(extra)
    span[1].record(stream)
    for b in range(nbuf):
        if pending[b] is not None:
            pending[b].wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    enqueue_us = (t_enq - t0) / a.steps * 1e6
    span_ms = span[0].elapsed_time(span[1]) / a.steps
    if a.kernel_steps > 0:
        kern_ms = time_launches(launch[0], a.kernel_steps, stream, preload="self") / 1e3
    else:
        kern_ms = span_ms

    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])

    # Parity (outside the timed region): every rank checks the buffers its timed steps wrote against
    # the oracle on the same input rows; rank 0 at N = 1 adds the one-shot configs A, B, C-SSD, D, E.
    parity = None
    if not a.no_parity:
        torch.cuda.synchronize()
        parity = parity_checks(dev, L[i0:i1], R[i0:i1], D, w,
                               [(disp_bufs[b][0, :rows], dist_bufs[b] if with_dist else None) for b in range(nbuf)],
                               one_shots=(world == 1 and rank == 0))
        bad = torch.tensor([0 if parity["ok"] else 1], dtype=torch.int64, device=dev)
        if world > 1:
            dist.all_reduce(bad, op=dist.ReduceOp.SUM)
        parity["ranks_with_mismatches"] = int(bad.item())
        parity["ok"] = parity["ranks_with_mismatches"] == 0

    pixels = W * H
    # bands: the job is one frame per step whatever N is; pairs: one frame per GPU per step
    value = (1 if bands else world) * a.steps * pixels / elapsed
    bytes_per_px = 3 + (8 if with_dist else 0)  # L + R + u8 disparity (+ f64 distance)
    alg_bytes = bytes_per_px * rows * W  # this rank's launch (its halo'd band when split by bands)
    achieved_gbs = alg_bytes / (kern_ms * 1e-3) / 1e9
    workload_key = f"{_config_name(W, H, w, D)}_{W}x{H}_w{w}_D{D}_{'dist' if with_dist else 'nodist'}"
    prof = None if bands else profile_counters(workload_key)  # counters were taken on whole frames
    kname = fast_kernel_name(W, D, w, W)
    rec = {
        "metric": BASELINE_METRIC,
        "value": value,
        "unit": "disparity-pixels/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "clock_warmup": {"ms": a.warm_ms, "untimed_steps": warm_steps},
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if bands else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded uniform u8 L, slab-shifted R with +-2 noise; SURVEY.md 8(d))",
        "config": {
            "workload": f"{_config_name(W, H, w, D)}: {W}x{H} u8 rectified pair, {w}x{w} SAD, D={D}, argmin u8 disparity"
                        + (" + fused f64 distance map (P/DistanceCalculator.cpp:84)" if with_dist else ""),
            "pairs_per_step": 1 if bands else world,
            "parallelism": (f"one frame in {world} row bands with {w // 2}-row halos, rank-0 RCCL gather of u8 "
                            f"disparity ({a.gather})" if bands else
                            f"one pair per GPU, rank-0 RCCL gather of u8 disparity ({a.gather})")
                           if world > 1 else "single GPU",
        },
        "disparity_evals_per_s": value * D,
        "kernel_ms": kern_ms,
        "kernel_timing": (f"HIP events around {a.kernel_steps} back-to-back launches after the timed region, "
                          f"enqueued behind {a.kernel_steps} untimed launches of the same kernel (so the host's "
                          "enqueue time is hidden) after 10 ms of warm launches, kernel's stream"
                          if a.kernel_steps > 0 else "HIP events around the timed region, span / steps"),
        "span_ms_per_step": span_ms,
        "host_enqueue_us_per_step": enqueue_us,
        "streams": len(streams),
        "stream_note": ("consecutive steps (independent frames) alternate over %d HIP streams, so a launch's "
                        "tail overlaps the next launch's head; kernel_ms is one launch alone" % len(streams)
                        if len(streams) > 1 else "one stream: launches strictly back to back"),
        "roofline": {
            "bound": "hbm",
            "achieved": achieved_gbs,
            "achieved_timed_region": alg_bytes / (span_ms * 1e-3) / 1e9,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_gbs / HBM_PEAK_GBS,
            "traffic": prof.get("bytes_per_launch") if prof else None,
            "traffic_source": prof.get("source") if prof else None,
            "algorithmic_bytes_per_launch": alg_bytes,
            "kernel": kname,
            "kernel_avg_us_rocprof": prof["avg_ns"] / 1e3 if prof else None,
            "note": "HBM is not the binding roof: the fused kernel is VALU-integer bound "
                    "(SURVEY.md 8(d)); see valu_roofline",
        },
    }
    if prof and prof.get("valu_insts_per_launch"):
        lane_ops = prof["valu_insts_per_launch"] * 64  # wave64 VALU instructions -> lane-ops
        rec["valu_roofline"] = {
            "achieved_lane_ops_per_s": lane_ops / (kern_ms * 1e-3),
            "peak": VALU_PEAK_LANE_OPS,
            "frac": lane_ops / (kern_ms * 1e-3) / VALU_PEAK_LANE_OPS,
            "lane_ops_per_element": lane_ops / (pixels * D),
            "source": "SQ_INSTS_VALU per launch x 64 from profiles/counters.json, over this run's kernel time",
        }
    if world == 1 and rank == 0 and a.pipeline_steps > 0:
        rec["pipeline"] = {"workload": f"{W}x{H} BGR frames, synthetic calibration (5-term distortion)",
                           "note": "per-frame stages around the matcher, SURVEY.md 8(f) rows 1 and 3; "
                                   "HBM roofline per leg (algorithmic bytes / avg launch, HIP events)",
                           **pipeline_legs(dev, W, H, a.pipeline_steps)}
    if world == 1 and rank == 0 and a.extra_steps > 0:
        rec["e2e"] = e2e_leg(dev, L, R, D, w, a.extra_steps)
        rec["frame_chain"] = frame_chain_leg(dev, W, H, D, w, a.extra_steps)
        rec["frame_chain_fused"] = frame_chain_fused_leg(dev, W, H, D, w, a.extra_steps)
        rec["frame_chain_overlap"] = frame_chain_overlap_leg(dev, W, H, D, w, a.extra_steps)
        rec["fallbacks"] = fallback_legs(dev, L, R, D, w, max(2, a.extra_steps // 4))
        rec["matcher"] = matcher_leg(dev)
    if world == 1 and rank == 0 and not a.no_cpu_baseline:
        rec["cpu_baseline"] = cpu_baseline(L, R, D, w, a.cpu_seconds)
        rec["cpu_baseline"]["speedup"] = value / rec["cpu_baseline"]["value"]
        rec["cpu_naive"] = cpu_naive_configs()
    if parity is not None:
        rec["parity"] = parity
    if rank == 0:
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and not parity["ok"]:
        print("bench.py: PARITY FAILURE -- the timed kernel's output differs from the oracle "
              f"({json.dumps(parity)})", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()

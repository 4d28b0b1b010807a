"""bench.py's launch contract on CPU (no GPU needed).

`--gpus N` must never turn into a one-rank measurement: without a launcher
bench.py spawns the N ranks itself (torch.distributed.run as a child), with a
launcher WORLD_SIZE must equal N, and too few GPUs is an error.  The N-rank
plumbing (spawn, barriers, max over ranks, rank-0 JSON line) is rehearsed with
USV_BENCH_PLUMBING=1 over gloo, which runs no kernel and reports value null.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _run(args, **env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=e, cwd=ROOT, timeout=240)


def test_gpus2_spawns_two_ranks_plumbing():
    out = _run(["--gpus", "2", "--steps", "3", "--warmup", "1"], USV_BENCH_PLUMBING="1")
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 only
    rec = lines[0]
    assert rec["n_gpus"] == 2 and rec["max_rank_seen"] == 1 and rec["value"] is None


def test_gpus_more_than_visible_fails():
    import torch
    if torch.cuda.device_count() >= 2:
        return  # a real multi-GPU host: the spawn path is the measurement itself
    out = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert out.returncode != 0
    assert "GPU(s) visible" in out.stderr


def test_world_size_mismatch_fails():
    out = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               USV_BENCH_PLUMBING="1")
    assert out.returncode != 0 and "WORLD_SIZE" in (out.stderr + out.stdout)


def test_parity_mismatch_counts():
    """bench.py's parity checker counts disparity bytes and distance bits that differ from the oracle's
    (inf at d = 0 compares equal as bits; a NaN or a 1-ulp change counts)."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    lut = np.array([np.inf] + [1000.0 / d for d in range(1, 256)])
    ref = np.array([[0, 1, 2], [3, 255, 0]], dtype=np.uint8)
    got = ref.copy()
    dist = lut[ref]
    assert bench._mismatches(got, ref, dist, lut) == {"pixels": 6, "disparity_mismatches": 0, "distance_mismatches": 0}
    got[0, 1] = 2
    dist2 = dist.copy()
    dist2[1, 1] = np.nextafter(dist2[1, 1], 0)
    dist2[0, 0] = np.nan
    assert bench._mismatches(got, ref, dist2, lut) == {"pixels": 6, "disparity_mismatches": 1,
                                                        "distance_mismatches": 2}
    assert bench._mismatches(got, ref, None, lut) == {"pixels": 6, "disparity_mismatches": 1}

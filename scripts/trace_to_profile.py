#!/usr/bin/env python3
"""Commit a gpurun_out/<tag>/ run of scripts/gpu_bench_prof.sh (smoke, pytest -m gpu, bench, a
rocprofv3 --kernel-trace --stats pass) as evidence under profiles/<tag>/: kernel_stats.csv, the bench
JSON line, the GPU test log tail and a summary.md table of per-kernel rocprof times.

    python scripts/trace_to_profile.py <tag> [--note TEXT]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--note", default="")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    bench = None
    blog = os.path.join(src, "bench.log")
    if os.path.exists(blog):
        for line in open(blog):
            if line.startswith("{"):
                bench = json.loads(line)
        if bench is not None:
            with open(os.path.join(dst, "bench.json"), "w") as f:
                json.dump(bench, f)
                f.write("\n")
    plog = os.path.join(src, "pytest.log")
    if os.path.exists(plog):
        lines = open(plog).read().splitlines()
        with open(os.path.join(dst, "pytest_gpu_tail.log"), "w") as f:
            f.write("\n".join(lines[-15:]) + "\n")
    rows = list(csv.DictReader(open(stats)))
    out = [f"# rocprofv3 kernel trace — {a.tag}", ""]
    if a.note:
        out += [a.note, ""]
    out += ["`rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "
            "--extra-steps 0` (scripts/gpu_bench_prof.sh)", "",
            "| kernel | calls | avg µs | min µs | max µs |", "|---|---|---|---|---|"]
    for r in rows:
        out.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.2f} | "
                   f"{float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} |")
    if bench:
        out += ["", f"bench line (same call, separate run): value {bench['value']:.4g} {bench['unit']}, "
                f"ms_per_step {bench['ms_per_step']:.4f}, kernel_ms {bench.get('kernel_ms', float('nan')):.4f}"]
        pipe = bench.get("pipeline", {})
        for k, v in pipe.items():
            if isinstance(v, dict) and "us" in v:
                out.append(f"- pipeline `{k}`: {v['us']:.2f} µs, {v['frac_hbm'] * 100:.1f} % of 8 TB/s")
    with open(os.path.join(dst, "summary.md"), "w") as f:
        f.write("\n".join(out) + "\n")
    print("wrote", dst)


if __name__ == "__main__":
    main()

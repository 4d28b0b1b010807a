#!/usr/bin/env python3
"""Turn a gpurun_out/prof_<tag>/ rocprofv3 run (scripts/profile.sh) into the
committed evidence under profiles/<tag>/ and the per-workload counter table
profiles/counters.json that bench.py reads for roofline.traffic.

    python scripts/summarize_profile.py <tag> [--workload KEY] [--kernel SUBSTR]

HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes and are in KiB.  The guide's x2
FETCH correction is calibrated for 16-B/lane streaming reads; for other access
widths it says to calibrate on a known byte count.  This kernel reads with
1-B LDS-DMA and scalar loads, and --fetch-factor records the calibration used
(see profiles/README.md: raw FETCH_SIZE equals the compulsory L+R bytes, and
the x2 reading of the no-remap build exceeds the 8-XCD upper bound).
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_stats(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counters(pass_dir, kernel_substr):
    """counter name -> median per-dispatch value over dispatches of the kernel."""
    out = {}
    for fn in os.listdir(pass_dir):
        if not fn.endswith("counter_collection.csv"):
            continue
        per = defaultdict(list)
        with open(os.path.join(pass_dir, fn)) as f:
            for row in csv.DictReader(f):
                if kernel_substr in row["Kernel_Name"]:
                    per[row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, v in per.items():
            out[k] = statistics.median(v)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--workload", default="C_1920x1080_w11_D128_dist")
    ap.add_argument("--kernel", default="sad_fast_kernel")
    ap.add_argument("--src", default=None, help="default gpurun_out/prof_<tag>")
    ap.add_argument("--fetch-factor", type=float, default=1.0,
                    help="FETCH_SIZE calibration (guide: 2 for 16-B/lane streaming reads)")
    a = ap.parse_args()
    src = a.src or os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}")
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)

    stats_csv = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats_csv, os.path.join(dst, "kernel_stats.csv"))
    stats = kernel_stats(stats_csv)
    dom = next(r for r in stats if a.kernel in r["Name"])
    avg_ns = float(dom["AverageNs"])

    c = {}
    for p in sorted(os.listdir(src)):
        d = os.path.join(src, p)
        if p.startswith("pmc_") and os.path.isdir(d):
            got = counters(d, a.kernel)
            if p.startswith("pmc_cold_"):  # cold-cache launches (scripts/prof_cold.py)
                got = {k + "_cold": v for k, v in got.items()}
            c.update(got)
            if got:
                shutil.copy(next(os.path.join(d, f) for f in os.listdir(d) if f.endswith("counter_collection.csv")),
                            os.path.join(dst, f"{p}.csv"))

    # HBM bytes: the cold-cache passes when present (inputs evicted before every launch), else the
    # bench's back-to-back launches (inputs may stay in L2 / Infinity Cache between launches)
    cold = "FETCH_SIZE_cold" in c and "WRITE_SIZE_cold" in c
    fk, wk = ("FETCH_SIZE_cold", "WRITE_SIZE_cold") if cold else ("FETCH_SIZE", "WRITE_SIZE")
    fetch_b = c.get(fk, 0.0) * 1024 * a.fetch_factor  # KiB -> B, calibrated
    # read requests by size (cold pass): exact for every load form (profiles/probes_r04/traffic_calibration_r04.md)
    sized = cold and all(f"TCC_EA0_RDREQ_{z}B_sum_cold" in c for z in (32, 64, 128))
    if sized:
        fetch_b = sum(z * c[f"TCC_EA0_RDREQ_{z}B_sum_cold"] for z in (32, 64, 128))
    how = ("32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B" if sized else f"{a.fetch_factor:g} x {fk}")
    write_b = c.get(wk, 0.0) * 1024
    hbm = fetch_b + write_b if fk in c and wk in c else None
    entry = {
        "kernel": dom["Name"],
        "avg_ns": avg_ns,
        "calls": int(dom["Calls"]),
        "fetch_bytes_per_launch": fetch_b if fk in c else None,
        "fetch_size_kib_raw": c.get(fk),
        "cache_state": "cold (512 MiB write between launches)" if cold else "warm (back-to-back bench launches)",
        "fetch_factor": None if sized else a.fetch_factor,
        "fetch_method": how,
        "write_bytes_per_launch": write_b if wk in c else None,
        "bytes_per_launch": hbm,
        "valu_insts_per_launch": c.get("SQ_INSTS_VALU"),
        "counters": c,
        "source": f"profiles/{a.tag}/ (rocprofv3 --kernel-trace --stats; separate --pmc passes; "
                  f"read bytes = {how}, write bytes = WRITE_SIZE KiB x 1024, "
                  f"{'cold-cache launches' if cold else 'bench launches'}; calibration in "
                  f"profiles/probes_r04/traffic_calibration_r04.md)",
    }
    table = os.path.join(ROOT, "profiles", "counters.json")
    allc = json.load(open(table)) if os.path.exists(table) else {}
    allc[a.workload] = entry
    json.dump(allc, open(table, "w"), indent=1, sort_keys=True)

    lines = [f"# rocprofv3 summary — {a.tag}", "", f"workload `{a.workload}`", "",
             "| kernel | calls | avg µs | min µs | max µs | % |", "|---|---|---|---|---|---|"]
    for r in stats:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | "
                     f"{float(r['MinNs'])/1e3:.2f} | {float(r['MaxNs'])/1e3:.2f} | {float(r['Percentage']):.1f} |")
    lines += ["", f"Dominant kernel per-launch counters (median over dispatches, `{a.kernel}`):", "",
              "| counter | value |", "|---|---|"]
    for k in sorted(c):
        lines.append(f"| {k} | {c[k]:.6g} |")
    if hbm is not None:
        lines += ["", f"HBM bytes per launch ({'cold' if cold else 'warm'}) = {how} + {wk} = {hbm/1e6:.2f} MB "
                      f"({hbm / (avg_ns * 1e-9) / 1e9:.0f} GB/s over the {avg_ns/1e3:.1f} µs average)"]
    if c.get("SQ_INSTS_VALU"):
        lane_ops = c["SQ_INSTS_VALU"] * 64
        lines += [f"VALU: {c['SQ_INSTS_VALU']:.4g} wave-instructions per launch = "
                  f"{lane_ops / (avg_ns * 1e-9) / 1e12:.1f} T lane-ops/s "
                  f"({lane_ops / (avg_ns * 1e-9) / (256 * 4 * 32 * 2.4e9) * 100:.0f}% of 78.6 T)"]
    open(os.path.join(dst, "summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()

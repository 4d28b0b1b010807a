#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration from scripts/gpu_traffic_probe.sh's passes
(gpurun_out/traffic/{fetch,write,rdreq}): per probe kernel, the median per-dispatch counter over its
launches against the 64 MiB it moved, written to profiles/probes_r04/traffic_calibration_r04.md."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "traffic")
BYTES = 64 << 20
FORMS = {
    "rd_vload_x4": "global_load_dwordx4 to VGPRs, 16 B per lane (the guide's reference form)",
    "rd_glds_x4": "global_load_lds_dwordx4, 16 B per lane (distance-table staging)",
    "rd_glds_ubyte": "global_load_lds_ubyte, 1 B per lane, 64 consecutive bytes per instruction",
    "rd_buf_ubyte": "buffer_load_ubyte ... lds (the paired kernel's steady-state R-row DMA)",
    "rd_sload_x8": "s_load_dwordx8, 32 B per wave instruction, each wave a contiguous 4 KiB (L-row segment form)",
    "wr_store_x4": "global_store_dwordx4, 16 B per lane",
    "wr_store_b64": "global_store_dwordx2, 8 B per lane (disparity flush store)",
}


def per_kernel(pass_name):
    out = defaultdict(lambda: defaultdict(list))
    for fn in glob.glob(os.path.join(SRC, pass_name, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            name = row["Kernel_Name"]
            for k in FORMS:
                if k in name:
                    out[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: statistics.median(v) for c, v in d.items()} for k, d in out.items()}


fetch, write, rdreq = per_kernel("fetch"), per_kernel("write"), per_kernel("rdreq")
lines = ["# FETCH_SIZE / WRITE_SIZE calibration (round 4)", "",
         "`scripts/probes/traffic_probe.hip` under `scripts/gpu_traffic_probe.sh`: every probe kernel moves exactly "
         f"{BYTES >> 20} MiB once, after a 512 MiB write that evicts the L2s and the Infinity Cache; counters are the "
         "median per-dispatch value over 3 launches (rocprofv3 --pmc, one counter per pass).  factor = bytes moved / "
         "(counter KiB x 1024).  The request-size counters resolve the form dependence: sized bytes = "
         "32 x RDREQ_32B + 64 x RDREQ_64B + 128 x RDREQ_128B (the L2-to-fabric read requests by size).", "",
         "| kernel | form | FETCH_SIZE KiB | fetch factor | WRITE_SIZE KiB | write factor | RDREQ | RDREQ 32B / 64B / 128B | sized read bytes / moved |",
         "|---|---|---|---|---|---|---|---|---|"]


def sized(rq, k):
    if "TCC_EA0_RDREQ_128B_sum" not in rq or not k.startswith("rd"):
        return "—"
    b = 32 * rq["TCC_EA0_RDREQ_32B_sum"] + 64 * rq["TCC_EA0_RDREQ_64B_sum"] + 128 * rq["TCC_EA0_RDREQ_128B_sum"]
    return f"{b / BYTES:.4f}"


for k, form in FORMS.items():
    f = fetch.get(k, {}).get("FETCH_SIZE")
    w = write.get(k, {}).get("WRITE_SIZE")
    rq = rdreq.get(k, {})
    ff = f"{BYTES / (f * 1024):.3f}" if f else "—"
    wf = f"{BYTES / (w * 1024):.3f}" if (w and k.startswith('wr')) else "—"
    lines.append(f"| `{k}` | {form} | {f if f is not None else '—'} | {ff} | {w if w is not None else '—'} | {wf} | "
                 f"{rq.get('TCC_EA0_RDREQ_sum', '—')} | {rq.get('TCC_EA0_RDREQ_32B_sum', '—')} / "
                 f"{rq.get('TCC_EA0_RDREQ_64B_sum', '—')} / {rq.get('TCC_EA0_RDREQ_128B_sum', '—')} | {sized(rq, k)} |")
lines += ["", "Reading: FETCH_SIZE counts 64 B per read request whatever its size (vector reads go out as 128-B "
          "requests, so FETCH_SIZE is half the bytes and the guide's x2 applies; scalar s_load lines go out as 64-B "
          "requests and FETCH_SIZE is exact).  A kernel that mixes forms cannot use one factor; the sized sum is "
          "exact for every form here and is what scripts/summarize_profile.py uses when the cold RDREQ pass exists.  "
          "A first version of the scalar probe, whose adjacent 32-B reads came from waves on different XCDs, "
          "measured twice the bytes: each XCD's L2 fetched the shared line (real duplicated traffic, not a counter "
          "artifact)."]
txt = "\n".join(lines) + "\n"
dst = os.path.join(ROOT, "profiles", "probes_r04", "traffic_calibration_r04.md")
os.makedirs(os.path.dirname(dst), exist_ok=True)
open(dst, "w").write(txt)
print(txt)

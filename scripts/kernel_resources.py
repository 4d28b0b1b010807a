#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy-relevant resources of the in-tree libusv.so (CPU only):
unbundles each translation unit's gfx950 code object and reads the AMDGPU metadata note.

    python scripts/kernel_resources.py [substring ...]   (default: the block-match kernels)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(ROOT, "unsynchronized_stereo_vision_proj325_amd", "libusv.so")


def main():
    subs = sys.argv[1:] or ["sad_pair_kernel", "sad_group_kernel", "ssd_fast_kernel", "sad_fast_kernel"]
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, fat], check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(b"__CLANG_OFFLOAD_BUNDLE__"), data)]
        rows = []
        for n, a in enumerate(starts):
            b = starts[n + 1] if n + 1 < len(starts) else len(data)
            part, co = os.path.join(td, f"b{n}"), os.path.join(td, f"c{n}.co")
            open(part, "wb").write(data[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                           check=True)
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            for blk in notes.split("  - .agpr_count")[1:]:
                get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]
                name = get("name")
                if any(s in name for s in subs):
                    rows.append((name, get("vgpr_count"), get("agpr_count") if False else "",
                                 get("sgpr_count"), get("group_segment_fixed_size"), get("private_segment_fixed_size"),
                                 get("vgpr_spill_count"), get("sgpr_spill_count")))
    print("| kernel | VGPRs | SGPRs | LDS bytes | scratch | VGPR spills | SGPR spills |")
    print("|---|---|---|---|---|---|---|")
    for name, v, _, s, lds, priv, vs, ss in sorted(rows):
        short = re.sub(r"_ZN3usv12_GLOBAL__N_1\d+", "", name)[:60]
        print(f"| `{short}` | {v} | {s} | {lds} | {priv} | {vs} | {ss} |")


if __name__ == "__main__":
    main()

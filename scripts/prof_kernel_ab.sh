#!/bin/bash
# GPU box: per-kernel rocprof times (kernel trace, no counters) of bench.py under ARGS for the in-tree build
# and each ${VARIANTS_DIR:-build_variants}/*.so, ROUNDS times in rotation; prints avg / median / min of the
# kernels whose name contains ${KSUB:-sad_}.  For launch-bound shapes (configs A, B) where the bench's
# HIP-event kernel_ms measures the host enqueue rather than the kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/kab.txt; : > $out
for r in $(seq ${ROUNDS:-3}); do
  for v in default ${VARIANTS_DIR:-build_variants}/*.so; do
    n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
    d=gpurun_out/kab_${n}_$r
    USV_LIB_PATH=$lib timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $d -o k \
       -- python3 bench.py $ARGS > $d.log 2>&1 || { echo "FAILED $n"; exit 1; }
    python3 - "$n" "$d" "${KSUB:-sad_}" >> $out <<'PY'
import csv, glob, statistics, sys
n, d, sub = sys.argv[1:]
f = glob.glob(f"{d}/**/k_kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if sub in r["Kernel_Name"]]
t = t[len(t) // 4:]  # drop the clock warm-up quarter
print(n, round(statistics.mean(t), 3), round(statistics.median(t), 3), round(min(t), 3), len(t))
PY
    tail -1 $out
  done
done
python3 - <<'PY'
import collections, statistics
d = collections.defaultdict(list)
for line in open("gpurun_out/kab.txt"):
    n, avg, med, mn, cnt = line.split()
    d[n].append(float(med))
for n, v in sorted(d.items()):
    print(f"{n:14s} kernel median-of-medians {statistics.median(v):8.3f} us  ({len(v)} runs: {v})")
PY

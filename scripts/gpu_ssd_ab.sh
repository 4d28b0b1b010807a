#!/bin/bash
# GPU box: parity of build_variants/ssd*.so, then rocprof kernel times of the SSD fast kernel (scripts/prof_ssd.py)
# for the in-tree library and each variant, 3 rounds in rotation.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in build_variants/ssd*.so; do
  n=$(basename $v .so)
  USV_LIB_PATH=$PWD/$v timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread > gpurun_out/vp_$n.log 2>&1
  rc=$?; echo "parity $n: $(tail -1 gpurun_out/vp_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/vp_$n.log; exit $rc; }
done
: > gpurun_out/ssd_ab.txt
for r in 1 2 3; do
  for v in default build_variants/ssd*.so; do
    n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
    d=gpurun_out/ssdab_${n}_$r
    USV_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o k -- python3 scripts/prof_ssd.py \
        > $d.log 2>&1 || { echo "FAILED $n"; exit 1; }
    python3 - "$n" "$d" >> gpurun_out/ssd_ab.txt <<'PY'
import csv, glob, statistics, sys
n, d = sys.argv[1:]
f = glob.glob(f"{d}/**/k_kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "ssd_fast" in r["Kernel_Name"]]
t = t[len(t) // 4:]
print(n, round(statistics.median(t), 2), round(min(t), 2), len(t))
PY
    tail -1 gpurun_out/ssd_ab.txt
  done
done

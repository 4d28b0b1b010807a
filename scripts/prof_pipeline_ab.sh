#!/bin/bash
# GPU box: per-kernel times of the pipeline stages (rocprofv3 --kernel-trace --stats) for the
# in-tree build and each build_variants/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default ${VARIANTS_DIR:-build_variants}/*.so; do
  n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
  USV_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pp_$n -o pp --output-format csv \
     -- python3 scripts/prof_pipeline.py > gpurun_out/pp_$n.log 2>&1 || { echo "FAILED $n"; exit 1; }
  echo "== $n"
  python3 - "$n" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/pp_{sys.argv[1]}/**/pp_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "usv" in r["Name"]:
        print(f"  {r['Name'][:56]:56s} {float(r['AverageNs'])/1e3:8.2f} us")
PY
done

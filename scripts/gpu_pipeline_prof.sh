#!/bin/bash
# GPU box: pipeline-stage parity tests, then rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes of
# scripts/prof_pipeline.py (20 x rectify pair, frame prep, motion mask at 1080p).  Usage: <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${1:-pp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
step() {
  local name=$1 to=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
step pytest 400 python -u -m pytest tests/test_rectify.py tests/test_preproc.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step trace 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 scripts/prof_pipeline.py
step fetch 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 scripts/prof_pipeline.py
step write 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 scripts/prof_pipeline.py
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = glob.glob(f"{out}/trace/**/trace_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "usv" in r["Name"]:
        print(f"  {r['Name'][:60]:60s} {float(r['AverageNs'])/1e3:8.2f} us (min {float(r['MinNs'])/1e3:.2f})")
for pmc in ("fetch", "write"):
    g = glob.glob(f"{out}/{pmc}/**/*counter_collection.csv", recursive=True)
    if not g: continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(g[0])):
        acc[(r["Kernel_Name"][:50], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        if "usv" in k: print(f"  {pmc:5s} {k:50s} {c:12s} median {sorted(v)[len(v)//2]:10.1f} KiB")
PY
exit 0

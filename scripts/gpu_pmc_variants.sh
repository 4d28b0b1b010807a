#!/bin/bash
# GPU box: rocprofv3 kernel trace + three SQ counter passes of a short config-C bench run for the
# in-tree build and every build_variants/*.so; prints the SAD kernel's per-launch medians side by side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcv
mkdir -p $OUT
ARGS=${ARGS:---steps 10 --warmup 2 --no-cpu-baseline --extra-steps 0 --pipeline-steps 0 --kernel-steps 5}
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
G3="SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_FLAT SQ_INSTS_LDS"
for v in default build_variants/*.so; do
  n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
  for g in 1 2 3; do
    eval "C=\$G$g"
    USV_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/${n}_g$g -o pmc --output-format csv \
      -- python3 bench.py $ARGS > $OUT/${n}_g$g.log 2>&1 || { echo "FAILED $n g$g"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, collections, os
rows = collections.defaultdict(dict)
for f in glob.glob("gpurun_out/pmcv/*_g*/**/*counter_collection.csv", recursive=True):
    n = os.path.basename(f.split("/pmcv/")[1].split("/")[0]).rsplit("_g", 1)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "sad_pair" in r["Kernel_Name"] or "sad_fast" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for c, v in acc.items():
        rows[c][n] = sorted(v)[len(v) // 2]
names = sorted({n for d in rows.values() for n in d})
print(f"{'counter':24s}" + "".join(f"{n:>14s}" for n in names))
for c in sorted(rows):
    print(f"{c:24s}" + "".join(f"{rows[c].get(n, float('nan')):14.4g}" for n in names))
PY

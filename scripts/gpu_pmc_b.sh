#!/bin/bash
# GPU box: per-launch SQ counters of the config-B kernel for the in-tree build and each build_variants/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/pmcB; mkdir -p $OUT
ARGS=${ARGS:-"--steps 5 --warmup 2 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --kernel-steps 5 --width 640 --height 480 --disparities 64 --window 7"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA"
for v in default build_variants/*.so; do
  n=$(basename $v .so); lib=""; [ "$v" != default ] && lib=$PWD/$v
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    USV_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/${n}_$i -o p --output-format csv -- python3 bench.py $ARGS > $OUT/${n}_$i.log 2>&1 || { echo "FAILED $n $i"; exit 1; }
  done
done
python3 - <<'PY'
import csv, glob, os, statistics, collections
for d in sorted(set(p.rsplit('_', 1)[0] for p in glob.glob('gpurun_out/pmcB/*_[12]') if os.path.isdir(p))):
    vals = collections.defaultdict(list)
    for f in glob.glob(d + '_*/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if 'sad_' in r['Kernel_Name']:
                vals[r['Counter_Name']].append(float(r['Counter_Value']))
    print(os.path.basename(d), {k: f"{statistics.median(v):.4g}" for k, v in sorted(vals.items())})
PY

#!/bin/bash
# GPU box: kernel trace + SQ counter passes of the SSD kernels at config C (scripts/prof_ssd.py), one pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_ssd}; mkdir -p $OUT
K=${KERNEL:-matrix}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P2="SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_MISC"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 scripts/prof_ssd.py $K 100 > $OUT/trace.log 2>&1 || { echo "FAILED trace"; exit 1; }
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o p --output-format csv -- python3 scripts/prof_ssd.py $K 30 > $OUT/p$i.log 2>&1 || { echo "FAILED pass $i"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, statistics, collections, sys
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(out + '/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'ssd' in r['Kernel_Name']:
            vals[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(f"{k:28s} {statistics.median(v):.6g}")
for f in glob.glob(out + '/trace/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'ssd' in r['Name']:
            print('trace', r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3)
PY
exit 0

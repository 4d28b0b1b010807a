#!/bin/bash
# GPU box: PMC passes (one group each, --pmc only) over scripts/prof_pipeline.py, summarised per pipeline kernel
# by scripts/pmc_by_kernel.py.  Usage: scripts/prof_pipeline_pmc.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/ppmc_${1:-r04}
mkdir -p $OUT
export PP_ITERS=${PP_ITERS:-40}
pass() {  # pass <name> <counters...>
  local n=$1; shift
  echo "=== $n"
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $OUT/$n -o $n --output-format csv -- python3 scripts/prof_pipeline.py \
     > $OUT/$n.log 2>&1 || { echo "FAILED $n"; tail -5 $OUT/$n.log; exit 1; }
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 scripts/prof_pipeline.py \
   > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
pass inst SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES
pass cyc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM
pass ta TA_TA_BUSY_sum TA_BUFFER_COALESCED_READ_CYCLES_sum
pass ta2 TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
pass td TD_TD_BUSY_sum
pass tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
python3 scripts/pmc_by_kernel.py $OUT
exit 0

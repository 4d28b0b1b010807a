#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box).  Kernel trace + stats in
# one pass; every PMC group in its own pass (no tracing domains beside --pmc).
# Output: gpurun_out/prof_<tag>/...  Usage: scripts/profile.sh <tag> [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}; shift
ARGS=${*:---steps 20 --warmup 5 --no-cpu-baseline --extra-steps 0}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {  # run <name> <rocprofv3 args...>
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 240 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
     > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 3 $OUT/$name.log
  if fatal $rc || [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $name: stopping"; exit $rc; fi
}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_inst --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
run pmc_cyc --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
run pmc_cyc2 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_FLAT SQ_INSTS_LDS
run pmc_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT
run pmc_icache --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQC_DCACHE_HITS SQC_DCACHE_MISSES
# cold-cache passes (a 512 MiB write between launches, scripts/prof_cold.py): HBM bytes per launch
if [ -n "$COLD" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    n=pmc_cold_$(echo $c | tr 'A-Z' 'a-z')
    echo "=== $n ($(date +%T))"
    timeout -k 10 240 rocprofv3 --pmc $c -d $OUT/$n -o $n --output-format csv -- python3 scripts/prof_cold.py $COLD 10 \
       > $OUT/$n.log 2>&1 || { echo "FAILED $n"; exit 1; }
  done
  # read requests by size (L2 -> fabric): true read bytes = 32*n32 + 64*n64 + 128*n128
  n=pmc_cold_rdreq; echo "=== $n ($(date +%T))"
  timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
     -d $OUT/$n -o $n --output-format csv -- python3 scripts/prof_cold.py $COLD 10 > $OUT/$n.log 2>&1 || echo "optional pass $n failed"
fi
run pmc_fifo --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU2 SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT
exit 0

#!/bin/bash
# rocprofv3 kernel trace + HBM byte passes + instruction mix for configs B and E (GPU box).
# Usage: scripts/profile_configs.sh <tag-prefix>   -> gpurun_out/prof_<prefix>_B, _E
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
P=${1:-r02}
fatal() { case "$1" in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
run() {  # run <dir> <name> <bench args> -- <rocprofv3 args...>
  local out=$1 name=$2 args=$3; shift 3
  mkdir -p $out
  echo "=== $out/$name ($(date +%T))"
  timeout -k 10 240 rocprofv3 "$@" -d $out/$name -o $name --output-format csv -- python3 bench.py $args \
     > $out/$name.log 2>&1
  local rc=$?
  echo "=== rc=$rc"; tail -n 2 $out/$name.log
  if fatal $rc || [ $rc -ne 0 ]; then echo "FAILED rc=$rc in $out/$name: stopping"; exit $rc; fi
}
B="--width 640 --height 480 --disparities 64 --window 7 --steps 50 --warmup 5 --no-cpu-baseline --extra-steps 0 --pipeline-steps 0"
E="--width 3840 --height 2160 --disparities 256 --window 15 --steps 10 --warmup 2 --no-cpu-baseline --extra-steps 0 --pipeline-steps 0"
for cfg in B E; do
  args=${!cfg}
  out=gpurun_out/prof_${P}_$cfg
  run $out trace "$args" --kernel-trace --stats
  run $out pmc_fetch "$args" --pmc FETCH_SIZE
  run $out pmc_write "$args" --pmc WRITE_SIZE
  run $out pmc_inst "$args" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
  run $out pmc_cyc "$args" --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
done
exit 0

#!/bin/bash
# GPU box (round 5): the small probes (MFMA i8 operand maps, unaligned LDS reads / LDS-DMA), each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/${TAG:-r05probes}; mkdir -p $OUT
for p in mfma_i8_layout lds_unaligned; do
  echo "=== $p"
  timeout -k 10 60 ./scripts/probes/bin_$p > $OUT/$p.txt 2>&1; rc=$?
  cat $OUT/$p.txt
  [ $rc -ne 0 ] && { echo "probe $p rc=$rc: stopping"; exit $rc; }
done
exit 0

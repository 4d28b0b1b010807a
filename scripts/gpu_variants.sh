#!/bin/bash
# GPU box: parity subset of the SAD kernels for every build_variants/*.so (USV_LIB_PATH), then an
# interleaved A/B of the in-tree build and the variants on config C (and E when AB_E=1).
# Each GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
SEL=${SEL:-"configC or fixtures or ragged or border or pitched or batch or fused"}
for v in build_variants/*.so; do
  n=$(basename $v .so)
  echo "=== parity $n ($(date +%T))"
  USV_LIB_PATH=$PWD/$v timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
      --timeout 120 --timeout-method thread -k "$SEL" > gpurun_out/parity_$n.log 2>&1
  rc=$?; tail -2 gpurun_out/parity_$n.log
  if [ $rc -ne 0 ]; then echo "FAILED parity $n rc=$rc: stopping"; tail -30 gpurun_out/parity_$n.log; exit 1; fi
done
if [ "${AB_E:-0}" = 1 ]; then
  ROUNDS=${ROUNDS_E:-2} ARGS="--steps 20 --warmup 3 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --kernel-steps 20 --width 3840 --height 2160 --disparities 256 --window 15" \
    timeout -k 10 600 bash scripts/ab_interleaved.sh || exit $?
  cp gpurun_out/ab.txt gpurun_out/abE.txt
fi
ROUNDS=${ROUNDS:-3} ARGS="--steps 100 --warmup 10 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --kernel-steps 200" \
  timeout -k 10 600 bash scripts/ab_interleaved.sh

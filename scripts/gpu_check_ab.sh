#!/bin/bash
# GPU-box run: the validation steps of gpu_check.sh, then an interleaved A/B of build_variants/*.so on
# config C (and config E when AB_E=1).  Every GPU step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
if [ "${SKIP_CHECK:-0}" != 1 ]; then bash scripts/gpu_check.sh || exit $?; fi
if [ "${AB_E:-0}" = 1 ]; then
  ROUNDS=${ROUNDS_E:-2} ARGS="--steps 20 --warmup 3 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0 --width 3840 --height 2160 --disparities 256 --window 15" \
    timeout -k 10 600 bash scripts/ab_interleaved.sh || exit $?
  cp gpurun_out/ab.txt gpurun_out/abE.txt
fi
ROUNDS=${ROUNDS:-3} ARGS="--steps 200 --warmup 20 --no-cpu-baseline --pipeline-steps 0 --extra-steps 0" \
  timeout -k 10 600 bash scripts/ab_interleaved.sh

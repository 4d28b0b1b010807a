#!/bin/bash
# GPU box: interleaved timing A/B of build_variants/*.so on configs C and E WITHOUT parity (timing-only
# experiment builds whose results are wrong by design).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} ARGS="--steps 200 --warmup 20 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0" \
    bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/tab_C.txt || exit 1
ROUNDS=${ROUNDS:-3} ARGS="--steps 60 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --width 3840 --height 2160 --disparities 256 --window 15" \
    bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/tab_E.txt

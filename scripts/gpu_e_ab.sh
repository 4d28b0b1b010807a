#!/bin/bash
# GPU box: interleaved A/B of build_variants/*.so on config E only (no parity: weight-only variants).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} ARGS="--steps 60 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --width 3840 --height 2160 --disparities 256 --window 15" \
    bash scripts/ab_interleaved.sh

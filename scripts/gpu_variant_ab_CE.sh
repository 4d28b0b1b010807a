#!/bin/bash
# GPU box: scripts/gpu_variant_ab.sh on config C, then the same interleaved A/B on config E (no parity rerun).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_variant_ab.sh || exit 1
cp gpurun_out/ab.txt gpurun_out/ab_C.txt
ROUNDS=${ROUNDS_E:-3} ARGS="--steps 60 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --width 3840 --height 2160 --disparities 256 --window 15" \
    bash scripts/ab_interleaved.sh && cp gpurun_out/ab.txt gpurun_out/ab_E.txt

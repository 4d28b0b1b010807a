#!/bin/bash
# GPU box: rocprof kernel-time A/B of the grouped kernel variants (build_variants_g/) on configs B and A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
base="--steps 400 --warmup 20 --no-cpu-baseline --no-parity --extra-steps 0 --pipeline-steps 0 --kernel-steps 0"
VARIANTS_DIR=build_variants_g KSUB=sad_group ARGS="$base --width 640 --height 480 --disparities 64 --window 7" \
    bash scripts/prof_kernel_ab.sh && cp gpurun_out/kab.txt gpurun_out/kab_B.txt || exit 1
VARIANTS_DIR=build_variants_g KSUB=sad_group ARGS="$base --width 320 --height 240 --disparities 32 --window 5" \
    bash scripts/prof_kernel_ab.sh && cp gpurun_out/kab.txt gpurun_out/kab_A.txt

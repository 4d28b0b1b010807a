#!/bin/bash
# GPU box: paired-kernel variants (build_variants/, configs C and E), grouped-kernel variants
# (build_variants_g/, configs B and A).  The first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_variant_ab_CE.sh || exit 1
VARIANTS_DIR=build_variants_g bash scripts/gpu_variant_ab_AB.sh

#!/bin/bash
# GPU box: timing-only A/B of build_variants/ (C, E; no parity), then the rocprof A/B of the grouped-kernel
# variants (build_variants_g/, configs B and A).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROUNDS=2 bash scripts/gpu_timing_ab.sh || exit 1
ROUNDS=2 bash scripts/gpu_group_ab.sh

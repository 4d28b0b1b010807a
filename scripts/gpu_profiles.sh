#!/bin/bash
# GPU box: scripts/profile.sh (kernel trace + separate PMC passes) for configs C, B and E, tag prefix $1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P=${1:-r03}
base="--steps 20 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 20"
COLD="1920 1080 128 11" bash scripts/profile.sh ${P}_C $base || exit 1
COLD="640 480 64 7" bash scripts/profile.sh ${P}_B $base --pipeline-steps 0 --width 640 --height 480 --disparities 64 --window 7 || exit 1
COLD="3840 2160 256 15" bash scripts/profile.sh ${P}_E --steps 5 --warmup 2 --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 5 --pipeline-steps 0 \
    --width 3840 --height 2160 --disparities 256 --window 15 || exit 1
exit 0

#!/bin/bash
# GPU box: scripts/profile.sh (kernel trace + separate PMC passes) for configs C, B, E and A, tag prefix $1;
# CONFIGS picks a subset (default "C B E A").  --streams 1: launches back to back on one stream, so each
# trace interval is one launch alone (with the bench's default two streams a launch's interval also
# covers the time it shares the chip with its neighbour).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
P=${1:-r05}
base="--steps 20 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 20 --streams 1"
for c in ${CONFIGS:-C B E A}; do
  case $c in
    C) COLD="1920 1080 128 11" bash scripts/profile.sh ${P}_C $base || exit 1 ;;
    B) COLD="640 480 64 7" bash scripts/profile.sh ${P}_B $base --pipeline-steps 0 --width 640 --height 480 \
         --disparities 64 --window 7 || exit 1 ;;
    A) COLD="320 240 32 5" bash scripts/profile.sh ${P}_A $base --pipeline-steps 0 --width 320 --height 240 \
         --disparities 32 --window 5 || exit 1 ;;
    E) COLD="3840 2160 256 15" bash scripts/profile.sh ${P}_E --steps 5 --warmup 2 --no-cpu-baseline --no-parity \
         --extra-steps 0 --kernel-steps 5 --pipeline-steps 0 --streams 1 --width 3840 --height 2160 \
         --disparities 256 --window 15 || exit 1 ;;
  esac
done
exit 0

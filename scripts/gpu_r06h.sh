#!/bin/bash
# GPU box (round 6): band-weight variants at config C (interleaved A/B), the product's config C profile
# (scripts/gpu_profiles.sh -> gpurun_out/prof_r06_C) and the K = 16 variant's counters (same passes, no cold passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r06h; mkdir -p $OUT
if [ -z "$NO_AB" ]; then
  echo "=== ab C ($(date +%T))"
  ROUNDS=${ROUNDS_C:-4} timeout -k 10 700 bash scripts/ab_interleaved.sh > $OUT/ab_C.log 2>&1 || { tail -5 $OUT/ab_C.log; exit 1; }
  cp gpurun_out/ab.txt $OUT/ab_C.txt; tail -5 $OUT/ab_C.log
fi
echo "=== profile C ($(date +%T))"
CONFIGS=C timeout -k 10 400 bash scripts/gpu_profiles.sh r06 > $OUT/prof_C.log 2>&1 || { tail -5 $OUT/prof_C.log; exit 1; }
echo "=== profile C, K = 16 ($(date +%T))"
USV_LIB_PATH=$PWD/build_variants_k16/k16ra4.so timeout -k 10 400 bash scripts/profile.sh r06_C16 --steps 20 --warmup 5 \
  --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 20 --streams 1 > $OUT/prof_C16.log 2>&1 || { tail -5 $OUT/prof_C16.log; exit 1; }
exit 0

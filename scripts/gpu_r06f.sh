#!/bin/bash
# GPU box (round 6): interleaved A/Bs of the variants in build_variants/ at config C (5 rounds) and config E, the
# V-histogram variants in build_variants_hist/ under rocprofv3 (scripts/prof_pipeline_ab.sh) and the SSD variants in
# build_variants_ssd/ (scripts/gpu_ssd_ab.py).  The first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06f}; mkdir -p $OUT
EARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 20 --pipeline-steps 0 --width 3840 --height 2160 --disparities 256 --window 15"
echo "=== ab C ($(date +%T))"
ROUNDS=${ROUNDS_C:-5} timeout -k 10 600 bash scripts/ab_interleaved.sh > $OUT/ab_C.log 2>&1 || { tail -5 $OUT/ab_C.log; exit 1; }
cp gpurun_out/ab.txt $OUT/ab_C.txt; tail -3 $OUT/ab_C.log
echo "=== ab E ($(date +%T))"
ROUNDS=3 ARGS="$EARGS" timeout -k 10 600 bash scripts/ab_interleaved.sh > $OUT/ab_E.log 2>&1 || { tail -5 $OUT/ab_E.log; exit 1; }
cp gpurun_out/ab.txt $OUT/ab_E.txt; tail -3 $OUT/ab_E.log
if [ -d build_variants_hist ]; then
  echo "=== hist ($(date +%T))"
  VARIANTS_DIR=build_variants_hist timeout -k 10 400 bash scripts/prof_pipeline_ab.sh > $OUT/hist.log 2>&1 || { tail -5 $OUT/hist.log; exit 1; }
  grep -E "==|hist" $OUT/hist.log
fi
if [ -d build_variants_ssd ]; then
  echo "=== ssd ($(date +%T))"
  VARIANTS_DIR=build_variants_ssd timeout -k 10 400 python scripts/gpu_ssd_ab.py > $OUT/ssd_ab.txt 2>&1 || { tail -5 $OUT/ssd_ab.txt; exit 1; }
  tail -3 $OUT/ssd_ab.txt
fi
exit 0

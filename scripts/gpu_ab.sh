#!/bin/bash
# GPU box: interleaved A/B of build_variants/ at config C (+ the parity suite on $VT variants), the product's
# config C profile (scripts/gpu_profiles.sh) and the K = 16 variant's counters (no cold passes).  The raw rocprofv3
# output is summarised on the box (scripts/summarize_profile.py -> profiles/<tag>, copied under gpurun_out/$TAG) and
# then deleted: the raw traces exceed what gpurun copies back.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
P=${PTAG:-r06}   # profile tag: profiles/${P}_C, profiles/${P}_C16
PT="python -u -m pytest -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
for v in ${VT}; do
  echo "=== parity $v ($(date +%T))"
  USV_LIB_PATH=$PWD/${VARIANTS_DIR:-build_variants}/$v.so timeout -k 10 600 $PT tests/test_gpu_parity.py > $OUT/vt_$v.log 2>&1 || { tail -5 $OUT/vt_$v.log; exit 1; }
  tail -1 $OUT/vt_$v.log
done
if [ -z "$NO_AB" ]; then
  echo "=== ab C ($(date +%T))"
  ROUNDS=${ROUNDS_C:-4} timeout -k 10 700 bash scripts/ab_interleaved.sh > $OUT/ab_C.log 2>&1 || { tail -5 $OUT/ab_C.log; exit 1; }
  cp gpurun_out/ab.txt $OUT/ab_C.txt; tail -5 $OUT/ab_C.log
fi
if [ -z "$NO_PROF" ]; then
  if [ -z "$NO_PROF_C" ]; then
  echo "=== profile C ($(date +%T))"
  CONFIGS=C timeout -k 10 400 bash scripts/gpu_profiles.sh $P > $OUT/prof_C.log 2>&1 || { tail -5 $OUT/prof_C.log; exit 1; }
  python scripts/summarize_profile.py ${P}_C --kernel sad_pair_kernel > $OUT/sum_C.log 2>&1 || { tail -5 $OUT/sum_C.log; exit 1; }
  cp -r profiles/${P}_C $OUT/ && cp profiles/counters.json $OUT/counters.json && rm -rf gpurun_out/prof_${P}_C
  fi
  echo "=== profile C, K = 16 ($(date +%T))"
  C16=${C16:-build_variants_k16/k16ra4}; C16T=${C16T:-${P}_C16}   # K = 16 build profiled, its profile tag
  USV_LIB_PATH=$PWD/$C16.so timeout -k 10 400 bash scripts/profile.sh $C16T --steps 20 --warmup 5 \
    --no-cpu-baseline --no-parity --extra-steps 0 --kernel-steps 20 --streams 1 > $OUT/prof_C16.log 2>&1 || { tail -5 $OUT/prof_C16.log; exit 1; }
  python scripts/summarize_profile.py $C16T --kernel sad_pair16_kernel --workload C16_variant_$(basename $C16) > $OUT/sum_C16.log 2>&1 || { tail -5 $OUT/sum_C16.log; exit 1; }
  cp -r profiles/$C16T $OUT/ && cp profiles/counters.json $OUT/counters.json && rm -rf gpurun_out/prof_$C16T
  grep -E "avg|SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU |SQ_INSTS_SALU|SQ_INSTS_LDS " $OUT/$C16T/summary.md | head -20
fi
exit 0

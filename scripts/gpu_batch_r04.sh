#!/bin/bash
# GPU box, round-4 batch: FETCH calibration probe; GPU tests of the new host-side engines; paired-kernel
# parity + interleaved A/B (build_variants/); the packed-f32 HSV2BGR frame-prep variant's parity and
# per-kernel times (build_variants_pp/).  Every step has its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <cmd...>
  echo "=== $1 ($(date +%T))"; local n=$1; shift
  "$@" > gpurun_out/b_$n.log 2>&1; local rc=$?
  tail -n 6 gpurun_out/b_$n.log
  [ $rc -ne 0 ] && { echo "FAILED rc=$rc in $n: stopping"; exit $rc; }
  return 0
}
[ "${SKIP_PROBE:-0}" = 1 ] || step traffic bash scripts/gpu_traffic_probe.sh
step tests timeout -k 10 400 python -u -m pytest tests/test_gpu_contours.py tests/test_streaming.py tests/test_sharded_engine.py tests/test_rectify.py \
    -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step pair_ab env ROUNDS=${ROUNDS:-3} bash scripts/gpu_ab_pair.sh
if ls build_variants_pp/*.so > /dev/null 2>&1; then
  for v in build_variants_pp/*.so; do
    step "pp_parity_$(basename $v .so)" env USV_LIB_PATH=$PWD/$v timeout -k 10 300 python -u -m pytest tests/test_preproc.py \
        -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
  done
  step pp_ab env PP_ITERS=300 VARIANTS_DIR=build_variants_pp bash scripts/prof_pipeline_ab.sh
fi
exit 0
